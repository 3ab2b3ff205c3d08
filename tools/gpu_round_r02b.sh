set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err
for p in 16384 65536 131072 262144 524288 1048576 2097152; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --points $p --no-cpu-baseline --no-full-iteration >> $O/size_sweep.jsonl 2>> $O/size_sweep.err
done
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python tools/precision_sweep.py --json $O/precision_sweep_c5.json > $O/precision_sweep.log 2>&1
echo done
