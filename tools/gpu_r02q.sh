# GPU suite, default bench, tracking bench (GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r02q}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
python -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'],d['ms_per_step'],d['config']['full_iteration_ms'],d['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/track_bench.py --json $O/track_bench_m64.json > $O/track.log 2>&1 || { tail -10 $O/track.log; exit 1; }
tail -2 $O/track.log
echo done
