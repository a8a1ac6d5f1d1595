#!/bin/bash
# One GPU call: GPU suite, then the rollout A/B of the Philox round-key forms
# (liborx.so: keys computed at use; tools/ab_libs/keyshoist.so: hoisted) over
# C3, C5 (both separation-damage states), C2 and the C3 shards, then the bench.
#   gpurun -- bash tools/gpu_keys_ab.sh <tag>
set -uo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=3 --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; case $rc in 124|134|137|139) exit $rc;; esac
AB_SMALL=1 AB_C5=1 AB_C5SEP=1 timeout -k 10 500 python3 tools/ab_rollout.py optimax_rogue_amd/liborx.so tools/ab_libs/keyshoist.so --ticks=128 > $O/ab_keys.jsonl 2> $O/ab_keys.err
rc=$?; cut -c1-300 $O/ab_keys.jsonl; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-200 $O/bench.json; exit $rc
