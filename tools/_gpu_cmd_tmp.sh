set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 600 python -m pytest tests -q -m gpu --timeout 300 -x > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bench.log 2>&1
