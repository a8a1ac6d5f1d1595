set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 600 -x > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bench.log 2>&1
