# Kernel traces of track! frames (tools/descend_probe.py) for each given build
# under abr/ (bash tools/trace_descend_ab.sh TAG LIB...), summary per build.
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
for L in "$@"; do
  ( cd /tmp && export TMPDIR=/tmp FLASHSDF_LIB=$GRAFT_REPO_ROOT/abr/lib_$L.so && timeout -k 10 200 rocprofv3 --kernel-trace \
      --output-format csv -d $O/tr_$L -o run -- python3 $GRAFT_REPO_ROOT/tools/descend_probe.py --frames 3 \
      > $O/tr_$L.log 2>&1 ) || { echo TRACE FAILED; tail $O/tr_$L.log; exit 1; }
  echo "== $L"; grep loop $O/tr_$L.log
  python3 $GRAFT_REPO_ROOT/tools/descend_probe.py --trace $(ls $O/tr_$L/*/run_kernel_trace.csv $O/tr_$L/run_kernel_trace.csv 2>/dev/null | head -1) > $O/tr_$L.txt
  grep -E "step_kernel|reduce_tiles|pose_kernel|pass_kernel|span|idle|per frame" $O/tr_$L.txt
done
