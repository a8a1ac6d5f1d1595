# usage: bash tools/_gpu_pmc_ab.sh lib1.so[:K] lib2.so[:K] ...  (one SQ pass per library, 128-tick launches)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcab
cd /tmp && export TMPDIR=/tmp
n=0
for LK in "$@"; do
  n=$((n+1))
  L=${LK%%:*}; K=8; case "$LK" in *:*) K=${LK##*:};; esac
  ORX_PROF_TICKS=128 ORX_LIB_OVERRIDE=$R/$L timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES -d $R/gpurun_out/pmcab/p$n -o pmc --output-format csv -- python3 $R/tools/prof_rollout.py 65536 1 $K 1 > $R/gpurun_out/pmcab/log$n.txt 2>&1
  f=$(find $R/gpurun_out/pmcab/p$n -name "*counter_collection.csv" | head -1)
  echo "== $L K=$K" >> $R/gpurun_out/pmcab/summary.txt
  python3 $R/tools/pmc_summary.py $f rollout >> $R/gpurun_out/pmcab/summary.txt
done
cat $R/gpurun_out/pmcab/summary.txt
