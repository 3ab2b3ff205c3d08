# One GPU-box round (run under gpurun): -m gpu tests, the default bench line,
# optionally the rocprofv3 passes of tools/rocprof_round.sh. Writes gpurun_out/$1/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail $O/bench_default.err; exit 1; }
if [ "${PROF:-0}" = 1 ]; then
  bash tools/rocprof_round.sh ${1:-round} > $O/rocprof.log 2>&1 || { echo ROCPROF FAILED; tail $O/rocprof.log; exit 1; }
fi
echo done
