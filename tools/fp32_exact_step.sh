#!/bin/bash
# One-off GPU step: the fp32 bit-exact parity tests alone (gpurun_out/$1/fp32.log).
mkdir -p gpurun_out/$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32_exact.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$1/fp32.log 2>&1; rc=$?; tail -25 gpurun_out/$1/fp32.log; exit $rc
