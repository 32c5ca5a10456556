#!/bin/bash
# Quick GPU iteration: score parity tests, then a short bench (no CPU leg).
# Stops at the first step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-quick}; shift || true
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 15 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path "$@" > "$OUT/bench.log" 2>&1
rc=$?; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' "$OUT/bench.log"; tail -n 3 "$OUT/bench.log"; exit $rc
