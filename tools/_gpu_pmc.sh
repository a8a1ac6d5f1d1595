set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
export ORX_ROLLOUT=plain
n=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_WAIT_ANY SQ_INSTS_BRANCH"; do
  n=$((n+1))
  timeout -k 10 180 rocprofv3 --pmc $C -d $R/gpurun_out/pmc/p$n -o pmc --output-format csv -- python3 $R/tools/prof_rollout.py 65536 1 8 0 > $R/gpurun_out/pmc/log$n.txt 2>&1
done
for n in 1 2 3 4; do f=$(find $R/gpurun_out/pmc/p$n -name "*counter_collection.csv" | head -1); python3 $R/tools/pmc_summary.py $f rollout; done > $R/gpurun_out/pmc/summary.txt
