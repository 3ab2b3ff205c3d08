#!/bin/bash
# 2-way vs 4-way hull partition vs one wave per chunk at 2^18 / 2^19 points
#   bash tools/hpart2_ab.sh TAG   (needs ab/lib_base.so, ab/lib_hp2.so from `make dev`)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for n in 262144 524288; do
  timeout -k 10 400 python tools/ab_bench.py ab/lib_base.so --rounds 3 -- --no-full-iteration --points $n \
    > $O/onewave_$n.log 2>&1 || { tail $O/onewave_$n.log; exit 1; }
  FSDF_HPART_POINTS=1048576 timeout -k 10 400 python tools/ab_bench.py ab/lib_base.so ab/lib_hp2.so --rounds 3 -- \
    --no-full-iteration --points $n > $O/hpart_$n.log 2>&1 || { tail $O/hpart_$n.log; exit 1; }
  echo "== $n one wave per chunk"; tail -2 $O/onewave_$n.log
  echo "== $n partitioned (lib_base: 4-way, lib_hp2: 2-way)"; tail -3 $O/hpart_$n.log
done
