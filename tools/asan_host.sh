#!/bin/bash
# AddressSanitizer on the host code (CPU; no GPU): instrumented builds of
# csrc/hull.cpp + csrc/kinematics.cpp + csrc/rbf_host.cpp and oracle/flash_oracle.c, driven from
# Python with libasan preloaded. Exits non-zero on the first ASan report.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/build_asan
mkdir -p $B
g++ -O1 -g -fsanitize=address -fno-omit-frame-pointer -fPIC -shared -std=c++17 -I$R/include \
    $R/point-cloud-signed-distance_amd/csrc/hull.cpp $R/point-cloud-signed-distance_amd/csrc/kinematics.cpp \
    $R/point-cloud-signed-distance_amd/csrc/rbf_host.cpp \
    -o $B/libfsdf_host_asan.so
gcc -O1 -g -fsanitize=address -fno-omit-frame-pointer -fPIC -mfma -mavx2 -ffp-contract=off -fno-fast-math \
    -fopenmp -shared $R/oracle/flash_oracle.c -o $B/liboracle_asan.so -lm
LD_PRELOAD=$(gcc -print-file-name=libasan.so) ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \
    ASAN_HOST_LIB=$B/libfsdf_host_asan.so ASAN_ORACLE_LIB=$B/liboracle_asan.so \
    python3 $R/tools/asan_host.py
