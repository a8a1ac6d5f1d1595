set -e
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_rollout.py optimax_rogue_amd/liborx.so@ORX_ROLLOUT=pc ab/nofb.so@ORX_ROLLOUT=pc > gpurun_out/ab.log 2>&1
