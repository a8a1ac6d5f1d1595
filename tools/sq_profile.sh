#!/bin/bash
# SQ counters of the headline rollout kernel (C3, 65,536 games, 128 ticks),
# one rocprofv3 --pmc pass per counter over tools/prof_kernels.py, each under
# its own time limit; the chain stops at the first failure.
#   gpurun --timeout 900 -- bash tools/sq_profile.sh <tag>
set -euo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
: > $O/sq_summary.txt
for C in SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH \
         SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$C -o pmc --output-format csv \
    -- python3 $R/tools/prof_kernels.py > $O/$C.log 2>&1
  f=$(find $O/$C -name "pmc_counter_collection.csv" | head -1)
  python3 $R/tools/pmc_summary.py $f "rollout_kernel<8, 1, false>" >> $O/sq_summary.txt
done
cat $O/sq_summary.txt
