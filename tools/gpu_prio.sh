# Heavy-wave issue priority: interleaved A/B at 2^20 and 2^17 points.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-prio}
mkdir -p $O
L="ab/lib_P0.so ab/lib_C12.so ab/lib_C20.so ab/lib_S3.so ab/lib_S5.so"
timeout -k 10 600 python tools/ab_bench.py $L --rounds 3 -- --no-full-iteration > $O/ab_1m.log 2>&1 || { tail -20 $O/ab_1m.log; exit 1; }
tail -7 $O/ab_1m.log
timeout -k 10 600 python tools/ab_bench.py $L --rounds 3 -- --no-full-iteration --points 131072 > $O/ab_128k.log 2>&1 || { tail -20 $O/ab_128k.log; exit 1; }
tail -7 $O/ab_128k.log
echo done
