set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r01
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python $R/tools/prof_kernels.py > $O/stats.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python $R/tools/prof_kernels.py > $O/fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python $R/tools/prof_kernels.py > $O/write.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/req -o run --output-format csv -- python $R/tools/prof_kernels.py > $O/req.log 2>&1 || true
