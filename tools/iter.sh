#!/bin/bash
# One GPU iteration: all gpu tests, a short bench, then the ablation split
# (LDGPU_ABLATE 1 = no verify, 2 = no probe, 3 = neither).  Stops at the
# first failing step.  Usage: tools/iter.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-iter}; shift || true
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 3 "$OUT/tests.log"; [ $rc -eq 0 ] || { tail -n 40 "$OUT/tests.log"; exit $rc; }
for a in ${ABLATE_SET:-0 1 2 3}; do
  LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_ABLATE=$a timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path "$@" > "$OUT/ab$a.log" 2>&1 \
    || { rc=$?; echo "bench ablate=$a failed rc=$rc"; tail -5 "$OUT/ab$a.log"; exit $rc; }
  echo "ablate=$a $(grep -o '"kernel_ms": [0-9.]*' "$OUT/ab$a.log")"
done
