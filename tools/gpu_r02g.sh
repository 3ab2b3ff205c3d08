# Split pass: parity tests, full GPU suite, budget x size sweep (GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > $O/split_tests.log 2>&1 || { echo SPLIT TESTS FAILED; tail -40 $O/split_tests.log; exit 1; }
timeout -k 10 300 python tools/split_sweep.py --json $O/split_sweep.json > $O/split_sweep.log 2>&1 || { tail -20 $O/split_sweep.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/split_tests.log; tail -2 $O/gpu_tests.log; cat $O/split_sweep.log
echo done
