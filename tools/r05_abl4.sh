#!/bin/bash
# Round 5: config 4's time split on the narrow diagnostics build (n4diag):
# LDGPU_ABLATE bits 1 verify, 2 probe, 16 >=3-byte tests, 32 argmax,
# 64 filter-word loads, 128 window loads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_abl4; mkdir -p $O
for a in ${ABL:-0 1 2 16 32 66 194 226}; do
  LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_${LIB:-n4diag}.so LDGPU_ABLATE=$a timeout -k 10 300 python3 -u bench.py ${CFG:---config 4} --steps 10 --warmup 2 \
    --no-cpu-baseline --no-host-path --no-alt-paths > $O/abl.log 2>&1 || { echo "fail $a"; tail -5 $O/abl.log; exit 1; }
  echo "ablate=$a $(grep -o '"kernel_ms": [0-9.]*' $O/abl.log)"
done
