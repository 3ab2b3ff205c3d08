# Lane-divergent many-seed waves: GPU tests (main lib built with FSDF_LANE_SEEDS=4),
# interleaved A/B of thresholds, per-wave timeline and size sweep of L4.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02x
mkdir -p $O
bash tools/gpu_ab.sh r02x "ab/lib_L0.so ab/lib_L3.so ab/lib_L4.so ab/lib_L6.so" > $O/ab_all.log 2>&1 || { tail -30 $O/ab_all.log; exit 1; }
tail -8 $O/ab_all.log
FLASHSDF_LIB=$PWD/ab/lib_wtL4.so timeout -k 10 200 python tools/wave_times.py --json $O/wt_1m.json > $O/wt_1m.log 2>&1 &&
FLASHSDF_LIB=$PWD/ab/lib_wtL4.so timeout -k 10 200 python tools/wave_times.py --points 131072 --json $O/wt_128k.json > $O/wt_128k.log 2>&1 &&
for v in L0 L4; do FLASHSDF_LIB=$PWD/ab/lib_$v.so timeout -k 10 200 python tools/split_sweep.py --budgets 0 --json $O/sweep_$v.json > $O/sweep_$v.log 2>&1 || exit 1; done
echo done
