set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > $O/solver_tests.log 2>&1 || { tail -30 $O/solver_tests.log; exit 1; }
tail -2 $O/solver_tests.log
for r in 1 2; do
  for L in head nt1024 fuseat; do
    for M in m64 irb140; do
      echo "== $L $M"; FLASHSDF_LIB=$PWD/abr/lib_$L.so timeout -k 10 120 python tools/descend_probe.py --model $M --frames 7 2>&1 | grep loop || exit 1
    done
  done
done
