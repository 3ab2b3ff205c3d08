# Diagnostics of the pass kernel (GPU box): work counters, phase timing,
# per-wave timeline at two cloud sizes. Writes gpurun_out/$1/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-diag}
mkdir -p $O
timeout -k 10 200 python tools/profile_pass.py --variants shuffled-1-64-1 --json $O/stats.json > $O/stats.log 2>&1
FLASHSDF_LIB=$PWD/ab/lib_phase.so timeout -k 10 200 python tools/profile_pass.py --variants shuffled-1-64-1 --json $O/phase.json > $O/phase.log 2>&1
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/wave_times.py --json $O/wt_1m.json > $O/wt_1m.log 2>&1
FLASHSDF_LIB=$PWD/ab/lib_wt.so timeout -k 10 200 python tools/wave_times.py --points 131072 --json $O/wt_128k.json > $O/wt_128k.log 2>&1
echo done
