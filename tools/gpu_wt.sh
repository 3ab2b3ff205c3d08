# Per-wave timeline with phase times and event counts (diagnostic build ab/lib_wt.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wt}
mkdir -p $O
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/wave_times.py --json $O/wt_1m.json > $O/wt_1m.log 2>&1 &&
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/wave_times.py --points 131072 --json $O/wt_128k.json > $O/wt_128k.log 2>&1
echo done
