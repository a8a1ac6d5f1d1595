set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
n=0
for MODE in plain; do
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY" "SQ_WAIT_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"; do
  n=$((n+1))
  ORX_ROLLOUT=$MODE timeout -k 10 180 rocprofv3 --pmc $C -d $R/gpurun_out/pmc/p$n -o pmc --output-format csv -- python3 $R/tools/prof_rollout.py 65536 1 8 1 > $R/gpurun_out/pmc/log$n.txt 2>&1
  f=$(find $R/gpurun_out/pmc/p$n -name "*counter_collection.csv" | head -1)
  echo "== $MODE $C" >> $R/gpurun_out/pmc/summary.txt
  python3 $R/tools/pmc_summary.py $f rollout >> $R/gpurun_out/pmc/summary.txt
done
done
