#!/bin/bash
# Kernel trace (no PMC) of back-to-back passes at a strong-scaling shard size:
#   bash tools/trace_small.sh TAG POINTS   -> gpurun_out/TAG/trace_POINTS/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1/trace_$2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/step_trace.py \
  --points $2 --steps 40 > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
cut -d, -f1-6 $O/run_kernel_stats.csv | cut -c1-160
