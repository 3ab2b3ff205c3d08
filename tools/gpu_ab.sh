# GPU tests with the main library, then an interleaved A/B of ab/lib_*.so builds.
#   bash tools/gpu_ab.sh TAG "libA libB ..." [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
LIBS=$2
shift 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python tools/ab_bench.py $LIBS --rounds 3 -- --no-full-iteration "$@" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
echo done
