set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 300 python tools/split_diag.py > $O/split_diag.log 2>&1 || { tail -20 $O/split_diag.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/split_sweep.py --budgets 1 --points 131072 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
cat $O/split_diag.log
cat $(find $O/trace -name "run_kernel_stats.csv") | cut -d, -f1-8 | head -20
echo done
