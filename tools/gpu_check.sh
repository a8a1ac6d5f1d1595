#!/bin/bash
# One GPU call (gpurun): the GPU test suite, the bench command, and 2-rank
# torchrun rehearsals of bench.py (gloo for the gather, both ranks on cuda:0)
# in weak and strong scaling.  Every step is time-limited; the chain stops at
# the first failure.  Output: gpurun_out/<tag>/.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh <tag> [tests|notests] [rehearse]
set -euo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cut -c1-400 $O/bench.json
if [ "${3:-}" = rehearse ]; then
  for MODE in weak strong; do
    EXTRA=""
    [ $MODE = strong ] && EXTRA="--strong"
    # bench.py starts the two ranks itself (torch.distributed.run underneath)
    timeout -k 10 300 python3 bench.py --gpus 2 \
      --steps 10 --warmup 3 --dist-backend gloo --same-device $EXTRA \
      > $O/bench_2rank_gloo_$MODE.json 2> $O/bench_2rank_gloo_$MODE.err
    cut -c1-300 $O/bench_2rank_gloo_$MODE.json
  done
fi
