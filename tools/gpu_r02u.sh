set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02u
mkdir -p $O
bash tools/gpu_ab.sh r02u "ab/lib_P.so ab/lib_Q.so" > $O/ab_all.log 2>&1 || { tail -30 $O/ab_all.log; exit 1; }
tail -5 $O/ab_all.log
cd /tmp && export TMPDIR=/tmp
for v in P Q; do
  export FLASHSDF_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/w_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/w_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
