# Native RBF iteration: GPU suite, then full-iteration timings native vs composed.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02n}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python tools/iteration_bench.py --json $O/iterations.json > $O/iterations.log 2>&1 || { tail -20 $O/iterations.log; exit 1; }
cat $O/iterations.log
echo done
