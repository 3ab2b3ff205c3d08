# 32-point chunks for small clouds: GPU suite (main lib: half chunks up to 2^22
# points), size sweep of H0 (64) and H1 (32) chunk libraries, A/B at 2^20.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-half}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for v in H0 H1; do FLASHSDF_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python tools/split_sweep.py --budgets 0 --json $O/sweep_$v.json > $O/sweep_$v.log 2>&1 || exit 1; done
grep points $O/sweep_H0.log $O/sweep_H1.log
timeout -k 10 600 python tools/ab_bench.py ab/lib_H0.so ab/lib_H1.so --rounds 3 -- --no-full-iteration > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -3 $O/ab.log
echo done
