#!/bin/bash
# Round-3 GPU pass: selected gpu tests (-k PATTERN, "all" = every gpu test),
# then any number of bench runs given as quoted argument strings; each step
# under its own time limit, stopping at the first fault / abort / timeout.
#   tools/history/r03_run.sh TAG PATTERN ["bench args" ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; PAT=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PAT" != "none" ]; then
  K=(); [ "$PAT" != "all" ] && K=(-k "$PAT")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/tests.log" 2>&1
  rc=$?; tail -n 4 "$OUT/tests.log"
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; exit $rc; fi
fi
i=0
for a in "$@"; do
  i=$((i+1))
  echo "== bench $i: $a"
  timeout -k 10 600 python -u bench.py $a --json-out "$OUT/bench$i.json" > "$OUT/bench$i.log" 2>&1
  rc=$?; tail -c 1500 "$OUT/bench$i.log"; echo
  [ $rc -eq 0 ] || exit $rc
done
