#!/bin/bash
# One GPU call (round 5): the GPU test suite, the bench command, the
# character-mechanics stamps at the bench's shard shape and the dungeon-bank
# forms A/B.  Each step is time-limited; a fault, abort or time-out (exit
# 124 / 134 / 137 / 139) ends the call, a failing test or tool does not.
#   gpurun --timeout 1500 -- bash tools/gpu_r05.sh <tag> [steps...]
TAG=${1:?tag}; shift
STEPS=${*:-"pytest bench stamps banks env"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "step $2 ended with $1: stopping"; exit $1;; esac; }
for s in $STEPS; do
  case $s in
    pytest)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 \
        --timeout-method thread > $O/pytest.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -25 $O/pytest.log; fatal $rc pytest;;
    bench)
      timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
      rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; fatal $rc bench;;
    stamps)
      for c in c3_rpg c3; do
        ORX_ROLLOUT_LANES=32 STAMPS_CFG=$c timeout -k 10 120 python3 tools/stamps.py \
          tools/ab_libs/stamps.so 32768 128 > $O/stamps_${c}_32768.json 2> $O/stamps_$c.err
        rc=$?; echo "stamps $c rc=$rc"; fatal $rc stamps
      done;;
    banks)
      timeout -k 10 400 python3 tools/bank_forms.py > $O/bank_forms.jsonl 2> $O/bank_forms.err
      rc=$?; echo "banks rc=$rc"; fatal $rc banks;;
    env)
      C5_FORMS=env timeout -k 10 300 python3 tools/c5_forms.py > $O/env_forms.jsonl 2> $O/env_forms.err
      rc=$?; echo "env rc=$rc"; fatal $rc env;;
    envtests)
      timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -k "env_step or vecenv or VecEnv" \
        --timeout 120 --timeout-method thread > $O/envtests.log 2>&1
      rc=$?; echo "envtests rc=$rc"; tail -5 $O/envtests.log; fatal $rc envtests;;
    abenv)
      timeout -k 10 600 python3 tools/ab_env.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 \
        > $O/ab_env.jsonl 2> $O/ab_env.err
      rc=$?; echo "abenv rc=$rc"; cat $O/ab_env.jsonl; fatal $rc abenv;;
    replaytests)
      timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -k "step_n" \
        --timeout 120 --timeout-method thread > $O/replaytests.log 2>&1
      rc=$?; echo "replaytests rc=$rc"; tail -5 $O/replaytests.log; fatal $rc replaytests;;
    abreplay)
      timeout -k 10 600 python3 tools/ab_replay.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 > $O/ab_replay.jsonl 2> $O/ab_replay.err
      rc=$?; echo "abreplay rc=$rc"; cat $O/ab_replay.jsonl; fatal $rc abreplay;;
    abptr)
      timeout -k 10 500 python3 tools/ab_forms.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 > $O/ab_forms.jsonl 2> $O/ab_forms.err
      rc=$?; echo "abforms rc=$rc"; cat $O/ab_forms.jsonl; fatal $rc abforms
      timeout -k 10 500 python3 tools/ab_c5.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=2 > $O/ab_c5.jsonl 2> $O/ab_c5.err
      rc=$?; echo "abc5 rc=$rc"; cat $O/ab_c5.jsonl; fatal $rc abc5;;
    stamps5)
      for c in c5 c5sep; do
        STAMPS_CFG=$c timeout -k 10 120 python3 tools/stamps.py \
          tools/ab_libs/stamps.so 16384 128 > $O/stamps_${c}_16384.json 2> $O/stamps_$c.err
        rc=$?; echo "stamps $c rc=$rc"; fatal $rc stamps
      done;;
    abc5)
      timeout -k 10 600 python3 tools/ab_c5.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 > $O/ab_c5.jsonl 2> $O/ab_c5.err
      rc=$?; echo "abc5 rc=$rc"; cat $O/ab_c5.jsonl; fatal $rc abc5;;
    abstep)
      timeout -k 10 600 python3 tools/ab_step.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 > $O/ab_step.jsonl 2> $O/ab_step.err
      rc=$?; echo "abstep rc=$rc"; cat $O/ab_step.jsonl; fatal $rc abstep;;
    abenvstep)
      timeout -k 10 600 python3 tools/ab_env.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 > $O/ab_env.jsonl 2> $O/ab_env.err
      rc=$?; echo "abenv rc=$rc"; cat $O/ab_env.jsonl; fatal $rc abenv
      timeout -k 10 600 python3 tools/ab_step.py tools/ab_libs/base.so tools/ab_libs/ptr.so \
        --reps=3 > $O/ab_step.jsonl 2> $O/ab_step.err
      rc=$?; echo "abstep rc=$rc"; cat $O/ab_step.jsonl; fatal $rc abstep;;
    c5)
      timeout -k 10 400 python3 tools/c5_forms.py > $O/c5_forms.jsonl 2> $O/c5_forms.err
      rc=$?; echo "c5 rc=$rc"; fatal $rc c5;;
  esac
done
exit 0
