# Kernel-trace stats of bench.py for each library build (pose / reduce kernel durations):
#   bash tools/gpu_pose_prof.sh TAG "ab/lib_A.so ab/lib_B.so"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
for L in $2; do
  n=$(basename $L .so)
  FLASHSDF_LIB=$R/$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-full-iteration > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  f=$(find $O/$n -name '*kernel_stats.csv' | head -1)
  echo "== $n"; grep -E 'pose_kernel|pass_kernel|reduce_tiles' $f | cut -d, -f1-4 | cut -c1-60,200-
done
