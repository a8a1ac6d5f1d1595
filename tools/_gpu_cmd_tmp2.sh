set -e
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_rollout.py optimax_rogue_amd/liborx.so optimax_rogue_amd/liborx.so > gpurun_out/ab.log 2>&1
