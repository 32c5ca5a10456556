#!/bin/bash
# Score-kernel time attribution (diagnostics library): config-2 bench with
# LDGPU_ABLATE = 0 (full), 1 (no verify), 2 (no probe), 8 (no 1-/2-byte
# direct counts), 16 (no >= 3-byte tests), under rocprofv3 kernel-trace stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ablscore}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
for a in ${ABLATE_SET:-0 1 2 8 16 24}; do
  LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/a$a" -o run -- python3 -u bench.py --docs 4000000 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path "$@" > "$OUT/a$a.log" 2>&1 || { echo "ablate $a failed"; tail -3 "$OUT/a$a.log"; exit 1; }
  f=$(find "$OUT/a$a" -name "*kernel_stats.csv" | head -1)
  echo "ablate=$a"; grep -E "score_kernel" "$f" | cut -d, -f1,3,4 | sed 's/(ldgpu[^"]*//'
done
