# Independent full-size check, default bench, rocprof trace + PMC (GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_independent.py -x -v --timeout 500 --timeout-method thread > $O/indep.log 2>&1 || { echo INDEP FAILED; tail -40 $O/indep.log; exit 1; }
tail -3 $O/indep.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-300 $O/bench_default.json
STEPS=20 bash tools/rocprof_round.sh r02j > $O/rocprof.log 2>&1 || { tail -20 $O/rocprof.log; exit 1; }
echo done
