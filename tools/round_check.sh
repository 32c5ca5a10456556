#!/bin/bash
# Round-end pass on one GPU box: gpu tests + smoke, then the bench set
# (tools/bench_all.sh).  Each step under its own limit; stops at the first
# failure.  Usage: tools/round_check.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -n 3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$OUT/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -n 2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
tools/bench_all.sh "$TAG"
