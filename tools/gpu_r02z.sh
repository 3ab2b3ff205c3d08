# Block-major partials + two-level reduce: GPU tests (main lib block-major),
# interleaved A/B (R0 entry-major, R2 line tiles), WRITE_SIZE per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02zb
mkdir -p $O
bash tools/gpu_ab.sh r02zb "ab/lib_R0.so ab/lib_R2.so" > $O/ab_all.log 2>&1 || { tail -30 $O/ab_all.log; exit 1; }
tail -5 $O/ab_all.log
cd /tmp && export TMPDIR=/tmp
for v in R0 R2; do
  export FLASHSDF_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/w_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/w_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/t_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/t_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo done
