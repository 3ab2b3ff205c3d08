# Packed candidate-bound loop: GPU tests (main lib) + interleaved A/B vs the
# previous kernel (ab/lib_R2.so) + kernel trace of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02c}
mkdir -p $O
bash tools/gpu_ab.sh $(basename $O) "ab/lib_R2.so ab/lib_C1.so" > $O/ab_all.log 2>&1 || { tail -30 $O/ab_all.log; exit 1; }
tail -4 $O/ab_all.log
cd /tmp && export TMPDIR=/tmp
for v in R2 C1; do
  export FLASHSDF_LIB=$GRAFT_REPO_ROOT/ab/lib_$v.so
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/t_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/t_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo done
