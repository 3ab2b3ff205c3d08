# Interleaved A/B of ab/lib_*.so builds at 2^20 and 2^17 points (+ the
# independent full-size check with the first library).
#   bash tools/gpu_ab2.sh TAG "libA libB ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
LIBS=$2
FIRST=${LIBS%% *}
FLASHSDF_LIB=$PWD/$FIRST timeout -k 10 300 python -u -m pytest tests/test_gpu_independent.py -x -q --timeout 250 --timeout-method thread > $O/indep.log 2>&1 || { echo INDEP FAILED; tail -30 $O/indep.log; exit 1; }
tail -1 $O/indep.log
timeout -k 10 600 python tools/ab_bench.py $LIBS --rounds 3 -- --no-full-iteration > $O/ab_1m.log 2>&1 || { tail -20 $O/ab_1m.log; exit 1; }
timeout -k 10 600 python tools/ab_bench.py $LIBS --rounds 3 -- --no-full-iteration --points 131072 > $O/ab_128k.log 2>&1 || { tail -20 $O/ab_128k.log; exit 1; }
tail -3 $O/ab_1m.log; tail -3 $O/ab_128k.log
echo done
