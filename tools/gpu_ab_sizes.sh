# GPU suite (main library), then an interleaved A/B of ab/lib_*.so builds at 2^20
# and 2^17 points:  bash tools/gpu_ab_sizes.sh TAG "ab/lib_A.so ab/lib_B.so ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
L=$2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python tools/ab_bench.py $L --rounds 3 -- --no-full-iteration > $O/ab_1m.log 2>&1 || { tail -20 $O/ab_1m.log; exit 1; }
grep -A9 summary $O/ab_1m.log
timeout -k 10 600 python tools/ab_bench.py $L --rounds 3 -- --no-full-iteration --points 131072 > $O/ab_128k.log 2>&1 || { tail -20 $O/ab_128k.log; exit 1; }
grep -A9 summary $O/ab_128k.log
echo done
