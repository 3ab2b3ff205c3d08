#!/bin/bash
# Interleaved A/B of the 2-waves-per-chunk tier (FSDF_HPART2_POINTS=0 disables it)
#   bash tools/hpart_tier_ab.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for r in 1 2 3; do
  for n in 262144 327680 393216; do
    for lim in 0 1048576; do
      FSDF_HPART2_POINTS=$lim timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
        --no-full-iteration --points $n > $O/b.json 2>> $O/tier.err || { tail $O/tier.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b.json')); print($r, $n, 'two-way' if $lim else 'one-wave', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))" | tee -a $O/tier_ab.txt
    done
  done
done
