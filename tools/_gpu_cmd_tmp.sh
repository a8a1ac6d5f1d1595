set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH"
for v in "65536 1 8" "65536 3 8" "65536 1 0" "1048576 1 8"; do
  n=$(echo $v | tr ' ' _)
  timeout -k 10 120 rocprofv3 --pmc $P -d $R/gpurun_out/pmc2/$n -o run --output-format csv -- python $R/tools/prof_rollout.py $v > $R/gpurun_out/pmc2/$n.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/pmc2/kt_$n -o run --output-format csv -- python $R/tools/prof_rollout.py $v > $R/gpurun_out/pmc2/kt_$n.log 2>&1
done
