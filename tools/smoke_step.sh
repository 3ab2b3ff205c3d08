#!/bin/bash
# __graft_entry__.smoke() on the GPU box (no build: the in-tree .so files travel)
mkdir -p gpurun_out/$1
timeout -k 10 300 python -c "import __graft_entry__ as g; g._paths(); g.smoke()" > gpurun_out/$1/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/$1/smoke.log; exit $rc
