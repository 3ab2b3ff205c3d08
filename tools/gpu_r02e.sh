# Round-2 re-entry check on the GPU box: GPU tests, default bench, per-wave
# timelines at 1M and 128K points (diagnostic build ab/lib_wt.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/wave_times.py --json $O/wt_1m.json > $O/wt_1m.log 2>&1 || exit 1
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/wave_times.py --points 131072 --json $O/wt_128k.json > $O/wt_128k.log 2>&1 || exit 1
tail -3 $O/gpu_tests.log; cat $O/bench_default.json | cut -c1-400
echo done
