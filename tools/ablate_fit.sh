#!/bin/bash
# Emit-kernel time attribution (diagnostics library): fit bench with
# LDGPU_FIT_EMIT_ABLATE = 0 (full), 1 (no 2-/3-byte LDS hash), 2 (no block
# stores), 4 (no records), under rocprofv3 kernel-trace stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ablfit}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
for a in ${ABLATE_SET:-0 1 2 4}; do
  LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_EMIT_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/a$a" -o run -- python3 -u bench.py --mode fit --steps 1 --warmup 0 --no-cpu-baseline --fit-bytes 268435456 > "$OUT/a$a.log" 2>&1 || { echo "ablate $a failed"; tail -3 "$OUT/a$a.log"; exit 1; }
  f=$(find "$OUT/a$a" -name "*kernel_stats.csv" | head -1)
  echo "ablate=$a"; grep -E "emit_kernel|part2_kernel|reduce_kernel|merge_kernel" "$f" | cut -d, -f1,3,4 | sed 's/(ldgpu[^"]*//'
  grep -o '"count_ms": [0-9.]*' "$OUT/a$a.log"
done
