# full GPU suite on the main library, then counters + A/B of J (seed), L (old), M (seed + pose overlap)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu_ab3.sh r02p "ab/lib_M.so ab/lib_J.so ab/lib_L.so"
