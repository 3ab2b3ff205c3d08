#!/bin/bash
# Profiles bench.py's default workload with rocprofv3 (run on the GPU box):
#   1. kernel trace + stats          -> gpurun_out/prof/<tag>_trace
#   2. PMC FETCH_SIZE (own pass)     -> gpurun_out/prof/<tag>_fetch
#   3. PMC WRITE_SIZE (own pass)     -> gpurun_out/prof/<tag>_write
#   4. PMC SQ instruction/wait mix   -> gpurun_out/prof/<tag>_sq
# Counters are collected in their own runs, never with tracing domains.
set -e
TAG=${1:-r01}
STEPS=${STEPS:-20}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof
mkdir -p $OUT
# the timed bench passes only (the full-iteration passes write no per-point outputs), one pass at a time
# (--inflight 1): each launch alone on the device, so its duration is the kernel's own
ARGS="$R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-full-iteration --inflight 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_trace -o run -- python3 $ARGS > $OUT/${TAG}_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${TAG}_fetch -o run -- python3 $ARGS > $OUT/${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${TAG}_write -o run -- python3 $ARGS > $OUT/${TAG}_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/${TAG}_sq -o run -- python3 $ARGS > $OUT/${TAG}_sq.log 2>&1 || echo "sq pass failed (counter set?)"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/${TAG}_sq2 -o run -- python3 $ARGS > $OUT/${TAG}_sq2.log 2>&1 || echo "sq2 pass failed"
echo done
