# Regrouping experiment + VALU breakdown by marginal-cost ablation builds (GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 200 python tools/group_experiment.py --json $O/group.json > $O/group.log 2>&1 || { tail -20 $O/group.log; exit 1; }
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/group_experiment.py --json $O/group_wt.json > $O/group_wt.log 2>&1 || { tail -20 $O/group_wt.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in base scr2 stg2 cul2 noslow nored nost; do
  export FLASHSDF_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
cd $GRAFT_REPO_ROOT
cat $O/group.log $O/group_wt.log
echo done
