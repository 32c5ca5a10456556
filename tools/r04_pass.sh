#!/bin/bash
# Round-4 GPU pass: gpu tests matching PATTERN ("all" / "none"), then an A/B of
# library builds (LIBS, CFGS as tools/ab.sh), stopping at the first failure.
#   tools/r04_pass.sh TAG PATTERN
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; PAT=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PAT" != "none" ]; then
  K=(); [ "$PAT" != "all" ] && K=(-k "$PAT")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/tests.log" 2>&1
  rc=$?; tail -n 4 "$OUT/tests.log"
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; exit $rc; fi
fi
if [ -n "${LIBS:-}" ]; then
  tools/ab.sh | tee "$OUT/ab.txt"
fi
