set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/pt.log 2>&1
timeout -k 10 600 python tools/ab_rollout.py optimax_rogue_amd/liborx.so@ORX_ROLLOUT=pc optimax_rogue_amd/liborx.so@ORX_ROLLOUT=pc@OBS=0 > gpurun_out/ab.log 2>&1
