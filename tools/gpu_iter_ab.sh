# Interleaved A/B of full CostFunctor iterations (tools/iteration_bench.py)
# between library builds:  bash tools/gpu_iter_ab.sh TAG "ab/lib_A.so ab/lib_B.so"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for r in 1 2 3; do
  for L in $2; do
    FLASHSDF_LIB=$PWD/$L timeout -k 10 300 python tools/iteration_bench.py --iters 50 --json $O/$(basename $L .so)_r$r.json > $O/$(basename $L .so)_r$r.log 2>&1 || { tail -20 $O/$(basename $L .so)_r$r.log; exit 1; }
    echo "round $r $L: $(grep -i 'ms' $O/$(basename $L .so)_r$r.log | tr '\n' ' ' | cut -c1-400)"
  done
done
