#!/bin/bash
# One GPU call: A/B of the small-batch launches (C2, C3 stream shards, C5)
# across diagnostic builds, and the cycle stamps of C2 and C5.  Stops at the
# first failing step.
#   gpurun -- bash tools/gpu_ab_small.sh <tag> lib1 [lib2 ...]
set -uo pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_SMALL=1 AB_C5=1 timeout -k 10 400 python3 tools/ab_rollout.py "$@" --ticks=128 > $O/ab_small.jsonl 2> $O/ab_small.err
rc=$?; cut -c1-400 $O/ab_small.jsonl; [ $rc -ne 0 ] && exit $rc
if [ -f tools/ab_libs/stamps.so ]; then
  STAMPS_CFG=c2 timeout -k 10 120 python3 tools/stamps.py tools/ab_libs/stamps.so 4096 128 > $O/stamps_c2.json 2> $O/stamps_c2.err
  rc=$?; [ $rc -ne 0 ] && exit $rc
  STAMPS_CFG=c5 timeout -k 10 120 python3 tools/stamps.py tools/ab_libs/stamps.so 16384 128 > $O/stamps_c5.json 2> $O/stamps_c5.err
  rc=$?; [ $rc -ne 0 ] && exit $rc
  cut -c1-300 $O/stamps_c2.json
fi
exit 0
