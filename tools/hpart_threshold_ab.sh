#!/bin/bash
# Interleaved A/B of the hull-partitioned pass threshold (FSDF_HPART_POINTS)
# at cloud sizes above the default: bash tools/hpart_threshold_ab.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for r in 1 2 3; do
  for n in 196608 262144 393216; do
    for thr in 131072 1048576; do
      FSDF_HPART_POINTS=$thr timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
        --no-full-iteration --points $n > $O/b.json 2>> $O/hp.err || { tail $O/hp.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$O/b.json')); print($r, $n, $thr, round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))" | tee -a $O/hpart_ab.txt
    done
  done
done
