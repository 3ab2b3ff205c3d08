# eval counters per library, then tools/gpu_ab2.sh (A/B at 2^20 and 2^17).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for L in $2; do FLASHSDF_LIB=$PWD/$L timeout -k 10 120 python tools/eval_counts.py >> $O/counts.log 2>&1 || { tail -5 $O/counts.log; exit 1; }; done
grep '^{' $O/counts.log
bash tools/gpu_ab2.sh "$@"
