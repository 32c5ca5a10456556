#!/bin/bash
# Round 5: the whole GPU test suite (one process, per-test timeout), then
# smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_full; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 \
  || { tail -n 60 $O/tests.log; exit 1; }
tail -n 3 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -n 30 $O/smoke.log; exit 1; }
tail -n 2 $O/smoke.log
