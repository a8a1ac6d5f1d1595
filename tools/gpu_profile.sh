#!/bin/bash
# One GPU call (gpurun): GPU tests, the bench command, its rocprofv3 kernel
# trace and its two PMC traffic passes.  Every step is time-limited and the
# chain stops at the first failure.  Output: gpurun_out/<tag>/.
#   gpurun --timeout 1100 -- bash tools/gpu_profile.sh <tag> [tests|notests]
set -euo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5"
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1
  tail -3 $O/pytest.log
fi
timeout -k 10 300 $BENCH > $O/bench.json 2> $O/bench.err
cat $O/bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_under_trace.json 2> $O/trace.err
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/ktrace_summary.py $f > $O/kernel_trace_summary.txt
KNAME=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['kernel'])" $O/bench.json)
python3 $R/tools/ktrace_summary.py --span $f "$KNAME" 65536 2 >> $O/kernel_trace_summary.txt
cp $(find $O/trace -name "run_kernel_stats.csv" | head -1) $O/kernel_stats.csv
# the PMC passes need only the headline's dispatches (make_traffic.py reads
# those): without the extras and the CPU baseline, so a pass stays short
# (the extras' thousands of small dispatches under counter collection can
# run minutes without output)
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv \
  -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
  > $O/bench_under_fetch.json 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv \
  -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
  > $O/bench_under_write.json 2> $O/write.err
python3 $R/tools/make_traffic.py $O/fetch $O/write $O/traffic.json > /dev/null
cat $O/traffic.json | tail -16
