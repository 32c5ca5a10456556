#!/bin/bash
# FIT GPU pass: FIT + distributed parity tests, then the config-3-shaped fit bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-fit}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_fit.py tests/test_distributed.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 4 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" "$OUT/tests.log" | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --mode fit --steps 3 --warmup 1 "$@" > "$OUT/bench.log" 2>&1
rc=$?; tail -c 2500 "$OUT/bench.log"; exit $rc
