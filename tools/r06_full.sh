#!/bin/bash
# Round 6: the whole -m gpu suite + smoke (the driver's round-end checks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06full}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 3 $OUT/gpu_tests.log; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -n 2 $OUT/smoke.log; exit $rc
