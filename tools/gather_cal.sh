#!/bin/bash
# FETCH_SIZE calibration on known-byte kernels (tools/gather_cal.hip): one
# rocprofv3 pass per counter group, never combined with tracing.  Build the
# binary here first:  make -C tools gather_cal  (or hipcc line below).
# Usage: tools/gather_cal.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gathercal}
mkdir -p "$OUT"
export TMPDIR=/tmp
BIN=tools/bin/gather_cal
timeout -k 10 120 $BIN > "$OUT/plain.json" || { echo "plain run failed"; exit 1; }
cat "$OUT/plain.json"
for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  name=$(echo "$pass" | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$PWD/$OUT/$name" -o run -- $BIN > "$OUT/$name.log" 2>&1
  rc=$?; echo "$pass rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
done
python3 tools/gather_cal.py "$OUT"
