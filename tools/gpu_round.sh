#!/bin/bash
# One GPU call: the bench command, the small-batch A/B (tools/gpu_ab_small.sh
# with the given libraries) and the GPU test suite; each step time-limited.
# A step that faults, aborts or times out (exit 124 / 134 / 137 / 139) ends
# the call; a failing test or bench does not stop the later steps.
#   gpurun -- bash tools/gpu_round.sh <tag> [lib ...]
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "step $2 ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; fatal $rc bench
if [ $# -gt 0 ]; then
  bash tools/gpu_ab_small.sh $TAG "$@"
  rc=$?; echo "ab rc=$rc"; fatal $rc ab
fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log; fatal $rc pytest
exit 0
