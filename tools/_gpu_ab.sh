set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "$1" = "--test" ]; then
  shift
  timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 400 python tools/ab_rollout.py "$@" --ticks=128
