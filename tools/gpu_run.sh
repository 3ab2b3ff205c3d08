#!/bin/bash
# The one GPU-box launcher (run under gpurun). Steps run in the order given,
# each under its own time limit; the first failure ends the call.
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# Steps (outputs under gpurun_out/TAG/):
#   tests           pytest -m gpu (one process)
#   pytest:FILES    pytest of the given test files only (commas between files)  -> pytest.log
#   ktrace:ARGS     rocprofv3 --kernel-trace --stats of bench.py ARGS (commas = spaces) -> ktrace_N/ + summary
#   smoke           __graft_entry__.smoke() (no build: the in-tree .so files travel)  -> smoke.log
#   bench           bench.py default line            -> bench_default.json
#   bench:ARGS      bench.py with ARGS (commas = spaces), e.g. bench:--points,131072
#   prof            tools/rocprof_round.sh (kernel trace + PMC passes)
#   ab:LIBS         interleaved A/B of ab/lib_*.so builds (commas between libs)
#   abn:P:LIBS      bit-for-bit check + A/B at a P-point cloud
#   wt:LIB          per-wave timeline of a -DFSDF_WAVE_TIMES=1 build, 2^20 and 2^17 points
#   stats:LIBS      kernel work counters of each build (bench cloud; commas between libs)
#   abcheck:LIBS    bit-for-bit agreement of builds with the first (tools/ab_check.py)
#   lds:LIBS        PMC pass of each build: LDS instructions / bank conflicts / waits
#   pmc:NAME:CTRS   one PMC pass (commas between counters) of the product library
#   pmclib:LIBS:CTRS  one PMC pass per library build (commas between libs, '+' between counters)
#   sweep           bench.py at 2^16 .. 2^20 points           -> size_sweep.jsonl
#   configs         tools/bench_configs.py (BASELINE configs C2-C5, M64)
#   rehearse        bench.py N=2 on one GPU (gloo, both ranks on device 0)
#   shards          strong-scaling shards stepped alone at W = 1/2/4/8 (tools/spatial_shards.py) -> spatial_shards.jsonl
#   hsweep:MODEL:SIZES[:EXTRA]  partition tiers / planned pass against cloud size (tools/hpart_sweep.py; MODEL
#                   irb140 | arm_grid, SIZES and EXTRA arguments comma-separated) -> hpart_sweep_MODEL*.jsonl
#   inflight:SIZES[:EXTRA]  independent passes in flight (tools/inflight_probe.py)  -> inflight.jsonl
#   split:MODEL:N   speed-up of 2- / 4-wave chunk splits at N points (tools/split_speedup.py) -> split_speedup.jsonl
#   abdriver        the driver's exact bench command, interleaved twice: HEAD, round 4 (abr/r04, an extracted
#                   1ef061e tree built in-tree), HEAD --no-regroup; device telemetry around each; then the
#                   rocprofv3 kernel trace of the same command at HEAD                  -> abdriver/
#   c5sweep         BASELINE C5 precision sweep on the reference cloud (tools/precision_sweep.py) -> c5_sweep.json
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/gpu_tests.log; exit 1; }
      tail -1 $O/gpu_tests.log ;;
    pytest:*)
      F=${step#pytest:}; F=${F//,/ }
      timeout -k 10 600 python -u -m pytest $F -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
        || { echo PYTEST FAILED; tail -40 $O/pytest.log; exit 1; }
      tail -3 $O/pytest.log ;;
    ktrace:*)
      A=${step#ktrace:}; A=${A//,/ }; N=$(echo "$A" | tr -c 'a-zA-Z0-9' '_')
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $GRAFT_REPO_ROOT/$O/ktrace_$N -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 \
          --no-cpu-baseline --no-full-iteration $A > $GRAFT_REPO_ROOT/$O/ktrace_$N.log 2>&1 ) \
        || { echo KTRACE FAILED; tail $O/ktrace_$N.log; exit 1; }
      python3 -c "
import csv, glob
f = glob.glob('$O/ktrace_$N/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('$N', r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us')" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g._paths(); g.smoke()" > $O/smoke.log 2>&1 \
        || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
      tail -2 $O/smoke.log ;;
    bench)
      timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
        || { echo BENCH FAILED; tail $O/bench_default.err; exit 1; }
      cut -c1-400 $O/bench_default.json ;;
    bench:*)
      A=${step#bench:}; A=${A//,/ }; N=$(echo "$A" | tr -c 'a-zA-Z0-9' '_')
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $A > $O/bench_$N.json 2> $O/bench_$N.err \
        || { echo BENCH FAILED; tail $O/bench_$N.err; exit 1; }
      cut -c1-400 $O/bench_$N.json ;;
    prof)
      bash tools/rocprof_round.sh $TAG > $O/rocprof.log 2>&1 || { echo ROCPROF FAILED; tail $O/rocprof.log; exit 1; } ;;
    ab:*)
      L=${step#ab:}; L=${L//,/ }
      timeout -k 10 900 python tools/ab_bench.py $L --rounds 3 -- --no-full-iteration > $O/ab.log 2>&1 \
        || { tail -20 $O/ab.log; exit 1; }
      cat $O/ab.log ;;
    abn:*)
      # abn:POINTS:LIBS — the A/B and the bit-for-bit check at a given cloud size
      R=${step#abn:}; P=${R%%:*}; L=${R#*:}; L=${L//,/ }
      timeout -k 10 300 python tools/ab_check.py $L --points $P > $O/abcheck_$P.log 2>&1 \
        || { echo ABCHECK FAILED; tail -20 $O/abcheck_$P.log; exit 1; }
      tail -4 $O/abcheck_$P.log
      timeout -k 10 900 python tools/ab_bench.py $L --rounds 3 -- --no-full-iteration --points $P > $O/ab_$P.log 2>&1 \
        || { tail -20 $O/ab_$P.log; exit 1; }
      tail -6 $O/ab_$P.log ;;
    wt:*)
      LIB=${step#wt:}; N=$(basename $LIB .so)
      FLASHSDF_LIB=$PWD/$LIB timeout -k 10 200 python tools/wave_times.py --json $O/wt_${N}_1m.json > $O/wt_${N}_1m.log 2>&1 &&
      FLASHSDF_LIB=$PWD/$LIB timeout -k 10 200 python tools/wave_times.py --points 131072 --json $O/wt_${N}_128k.json \
        > $O/wt_${N}_128k.log 2>&1 || { echo WT FAILED; tail $O/wt_${N}_1m.log $O/wt_${N}_128k.log; exit 1; }
      echo "wt $N: $(cut -c1-200 $O/wt_${N}_1m.log)" ;;
    stats:*)
      L=${step#stats:}
      for lib in ${L//,/ }; do
        FLASHSDF_LIB=$PWD/$lib timeout -k 10 200 python tools/profile_pass.py --variants shuffled-1-64-1 --reps 3 \
          --rounds 2 >> $O/stats.log 2>&1 || { echo STATS FAILED; tail $O/stats.log; exit 1; }
        echo "$lib $(tail -1 $O/stats.log | cut -c1-700)"
      done ;;
    abcheck:*)
      L=${step#abcheck:}; L=${L//,/ }
      timeout -k 10 300 python tools/ab_check.py $L > $O/abcheck.log 2>&1 || { echo ABCHECK FAILED; tail -20 $O/abcheck.log; exit 1; }
      tail -5 $O/abcheck.log ;;
    lds:*)
      L=${step#lds:}
      for lib in ${L//,/ }; do
        N=$(basename $lib .so)
        ( cd /tmp && export TMPDIR=/tmp FLASHSDF_LIB=$GRAFT_REPO_ROOT/$lib && timeout -s KILL 120 rocprofv3 --pmc \
          SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU \
          --output-format csv -d $GRAFT_REPO_ROOT/$O/lds_$N -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 \
          --warmup 3 --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/lds_$N.log 2>&1 ) \
          || { echo LDS PMC FAILED; tail $O/lds_$N.log; exit 1; }
        python tools/pmc_brief.py $O/lds_$N/run_counter_collection.csv pass_kernel ;
      done ;;
    pmc:*)
      # pmc:NAME:C1,C2,... — one counter pass over the product library (<= 8 SQ counters)
      R=${step#pmc:}; N=${R%%:*}; C=${R#*:}; C=${C//,/ }
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv \
          -d $GRAFT_REPO_ROOT/$O/pmc_$N -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 \
          --no-cpu-baseline --no-full-iteration > $GRAFT_REPO_ROOT/$O/pmc_$N.log 2>&1 ) \
        || { echo PMC FAILED; tail $O/pmc_$N.log; exit 1; }
      python tools/pmc_brief.py $O/pmc_$N/run_counter_collection.csv pass_kernel ;;
    pmclib:*)
      # pmclib:LIBS:C1,C2,... — one PMC pass per library build (FLASHSDF_LIB; commas between libs, '+' between counters)
      R=${step#pmclib:}; L=${R%%:*}; C=${R#*:}; C=${C//+/ }
      for lib in ${L//,/ }; do
        N=$(basename $lib .so)
        ( cd /tmp && export TMPDIR=/tmp FLASHSDF_LIB=$GRAFT_REPO_ROOT/$lib && timeout -s KILL 120 rocprofv3 --pmc $C \
          --output-format csv -d $GRAFT_REPO_ROOT/$O/pmclib_$N -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 \
          --warmup 3 --no-cpu-baseline --no-full-iteration --inflight 1 > $GRAFT_REPO_ROOT/$O/pmclib_$N.log 2>&1 ) \
          || { echo PMCLIB FAILED; tail $O/pmclib_$N.log; exit 1; }
        echo "$N $(python tools/pmc_brief.py $O/pmclib_$N/run_counter_collection.csv pass_kernel)"
      done ;;
    sweep)
      # M64 pass/step against cloud size (one bench line per size)
      for n in 65536 131072 262144 524288 1048576; do
        timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-iteration --points $n \
          >> $O/size_sweep.jsonl 2>> $O/size_sweep.err || { echo SWEEP FAILED; tail $O/size_sweep.err; exit 1; }
      done
      cut -c1-200 $O/size_sweep.jsonl ;;
    configs)
      timeout -k 10 400 python tools/bench_configs.py --json $O/bench_configs.json > $O/bench_configs.log 2>&1 \
        || { echo CONFIGS FAILED; tail $O/bench_configs.log; exit 1; }
      tail -12 $O/bench_configs.log ;;
    rehearse)
      export FSDF_BENCH_BACKEND=gloo FSDF_BENCH_DEVICE=0
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 > $O/rehearse_n2.json 2> $O/rehearse_n2.err \
        || { tail -30 $O/rehearse_n2.err; exit 1; }
      cut -c1-600 $O/rehearse_n2.json
      unset FSDF_BENCH_BACKEND FSDF_BENCH_DEVICE ;;
    shards)
      # strong-scaling shards of the bench cloud, each stepped alone (tools/spatial_shards.py)
      timeout -k 10 600 python -u tools/spatial_shards.py > $O/spatial_shards.jsonl 2> $O/spatial_shards.err \
        || { echo SHARDS FAILED; tail $O/spatial_shards.err; exit 1; }
      cut -c1-200 $O/spatial_shards.jsonl ;;
    hsweep:*)
      # hsweep:MODEL:SIZES[:EXTRA] — EXTRA: more tools/hpart_sweep.py arguments, commas = spaces
      R=${step#hsweep:}; M=${R%%:*}; R=${R#*:}; S=${R%%:*}; X=""; [ "$R" != "$S" ] && X=${R#*:}; X=${X//,/ }
      N=$M$(echo "$X" | tr -c 'a-zA-Z0-9.' '_')
      timeout -k 10 600 python tools/hpart_sweep.py --model $M --sizes $S $X >> $O/hpart_sweep_$N.jsonl \
        2>> $O/hpart_sweep_$N.err || { echo HSWEEP FAILED; tail $O/hpart_sweep_$N.err; exit 1; }
      python3 -c "
import json
for l in open('$O/hpart_sweep_$N.jsonl'):
    d = json.loads(l); print(d['points'], d['tier'], d['shares'], round(d['step_ms'], 4), round(d['pass_kernel_ms'], 4), d['default_parts'])" ;;
    inflight:*)
      # inflight:SIZES[:EXTRA] — tools/inflight_probe.py (EXTRA: more arguments, commas = spaces)
      R=${step#inflight:}; S=${R%%:*}; X=""; [ "$R" != "$S" ] && X=${R#*:}; X=${X//,/ }
      timeout -k 10 300 python tools/inflight_probe.py --sizes $S $X >> $O/inflight.jsonl 2>> $O/inflight.err \
        || { echo INFLIGHT FAILED; tail $O/inflight.err; exit 1; }
      cat $O/inflight.jsonl ;;
    split:*)
      # split:MODEL:POINTS — measured speed-up of 2- / 4-wave chunk splits (tools/split_speedup.py)
      R=${step#split:}; M=${R%%:*}; P=${R#*:}
      timeout -k 10 300 python tools/split_speedup.py --model $M --points $P >> $O/split_speedup.jsonl \
        2>> $O/split_speedup.err || { echo SPLIT FAILED; tail $O/split_speedup.err; exit 1; }
      tail -1 $O/split_speedup.jsonl | cut -c1-600 ;;
    abdriver)
      D=$O/abdriver; mkdir -p $D
      CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5"
      TEL="import bench, json; print(json.dumps(bench.device_telemetry(0)))"
      for rep in 1 2; do
        timeout -k 10 300 $CMD > $D/head_$rep.json 2> $D/head_$rep.err || { echo AB HEAD FAILED; tail $D/head_$rep.err; exit 1; }
        ( timeout -k 10 60 python3 -c "$TEL" > $D/r04_${rep}_tel0.json && cd abr/r04 && timeout -k 10 300 $CMD ) \
          > $D/r04_$rep.json 2> $D/r04_$rep.err || { echo AB R04 FAILED; tail $D/r04_$rep.err; exit 1; }
        timeout -k 10 60 python3 -c "$TEL" > $D/r04_${rep}_tel1.json || exit 1
        timeout -k 10 300 $CMD --no-regroup > $D/noregroup_$rep.json 2> $D/noregroup_$rep.err \
          || { echo AB NOREGROUP FAILED; tail $D/noregroup_$rep.err; exit 1; }
        for f in head r04 noregroup; do python3 -c "
import json; d = json.load(open('$D/${f}_$rep.json')); c = d['config']; r = d['roofline']
print('$f $rep', round(d['value'] / 1e9, 3), 'G', round(d['ms_per_step'], 5), 'serial', round(c['serial_step_ms'], 5),
      'kernel', round(r['kernel_ms'], 5), 'frac', round(r['frac'], 4))"; done
      done
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $GRAFT_REPO_ROOT/$D/ktrace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 \
          > $GRAFT_REPO_ROOT/$D/ktrace.json 2> $GRAFT_REPO_ROOT/$D/ktrace.err ) || { echo AB KTRACE FAILED; tail $D/ktrace.err; exit 1; }
      python3 -c "
import csv, glob
f = glob.glob('$D/ktrace/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:4]:
    print('ktrace', r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 3), 'us')" ;;
    descend)
      # track! frames through fsdf_descend (device and host solver loops) under a kernel trace
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
          -d $GRAFT_REPO_ROOT/$O/descend -o run -- python3 $GRAFT_REPO_ROOT/tools/descend_probe.py \
          > $GRAFT_REPO_ROOT/$O/descend.log 2>&1 ) || { echo DESCEND FAILED; tail $O/descend.log; exit 1; }
      cat $O/descend.log
      python3 tools/descend_probe.py --trace $(ls $O/descend/*/run_kernel_trace.csv $O/descend/run_kernel_trace.csv 2>/dev/null | head -1) ;;
    c4proj)
      # BASELINE C4 projection from one GPU: per-pass and per-frame (ingest) max over ranks (tools/c4_projection.py)
      timeout -k 10 600 python -u tools/c4_projection.py > $O/c4_projection.jsonl 2> $O/c4_projection.err \
        || { echo C4PROJ FAILED; tail $O/c4_projection.err; exit 1; }
      cut -c1-300 $O/c4_projection.jsonl ;;
    c5sweep)
      timeout -k 10 300 python tools/precision_sweep.py --json $O/c5_sweep.json > $O/c5_sweep.log 2>&1 \
        || { echo C5 SWEEP FAILED; tail $O/c5_sweep.log; exit 1; }
      tail -5 $O/c5_sweep.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
