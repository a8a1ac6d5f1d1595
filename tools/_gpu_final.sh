set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu --timeout 300 -x > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/kt -o run --output-format csv -- python3 $R/bench.py --no-extras --no-cpu-baseline > $R/gpurun_out/prof/kt_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof/fetch -o pmc --output-format csv -- python3 $R/tools/prof_kernels.py > $R/gpurun_out/prof/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof/write -o pmc --output-format csv -- python3 $R/tools/prof_kernels.py > $R/gpurun_out/prof/write.log 2>&1
