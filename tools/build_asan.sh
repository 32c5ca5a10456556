#!/bin/bash
# Host-code AddressSanitizer build of libldgpu (lib/libldgpu_asan.so) and its
# driver (tools/bin/asan_driver, linking the C restatement as the checker).
# Built here on the CPU; run on a GPU box:
#   ASAN_OPTIONS=detect_leaks=0 tools/bin/asan_driver
set -eu
cd "$(dirname "$0")/.."
make -s -j8 -C spark-languagedetector_amd asan
mkdir -p tools/bin
/opt/rocm/llvm/bin/clang -O1 -g -fno-omit-frame-pointer -fsanitize=address -std=c11 \
    tools/asan_driver.c oracle/ldoracle.c \
    -Lspark-languagedetector_amd/lib -lldgpu_asan -L/opt/rocm/lib -lpthread \
    -Wl,-rpath,'$ORIGIN/../../spark-languagedetector_amd/lib' -Wl,-rpath,/opt/rocm/lib -o tools/bin/asan_driver
echo "built tools/bin/asan_driver"
