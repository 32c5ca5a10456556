#!/bin/bash
# Time attribution of the SCORE kernel (diagnostics library, make diag): bench with LDGPU_ABLATE = 0 (full),
# 1 (no verify/accumulate), 2 (no probe), 3 (staging + argmax only),
# 4 (no hit replay).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ablate}; shift || true
mkdir -p "$OUT"
for a in ${ABLATE_SET:-0 1 2 3}; do
  LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_ABLATE=$a timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path "$@" > "$OUT/ab$a.log" 2>&1 || { echo "ablate $a failed rc=$?"; tail -5 "$OUT/ab$a.log"; exit 1; }
  echo "ablate=$a $(grep -o '"kernel_ms": [0-9.]*' "$OUT/ab$a.log")"
done
