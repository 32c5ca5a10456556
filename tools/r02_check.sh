#!/bin/bash
# Round-2 GPU pass: gpu tests (verbose, per-test timeout) then the headline
# bench.  Stops at the first step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r02}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 5 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?; tail -c 3000 "$OUT/bench.log"; exit $rc
