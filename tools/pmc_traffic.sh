#!/bin/bash
# HBM traffic of the SCORE kernel from PMC counters (MI355X_MICROARCH.md §HBM):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (never combined with
# tracing), each over the real workload and over an empty-table calibration run
# whose bytes are known exactly (documents + offsets read, labels written),
# plus the L2 (TCC) hit / miss counts of the real workload.
# Writes $OUT/pmc_traffic.json (copy it to profiles/ to have bench.py report it).
# Usage: tools/pmc_traffic.sh <outdir> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name counter extra-args...
  local name=$1 ctr=$2; shift 2
  echo "== $name ($ctr)"
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/$name" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths --json-out "$PWD/$OUT/$name.json" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
run fetch_real FETCH_SIZE "$@"
run write_real WRITE_SIZE "$@"
run fetch_cal FETCH_SIZE --empty-table "$@"
run write_cal WRITE_SIZE --empty-table "$@"
run l2_real "TCC_HIT_sum TCC_MISS_sum" "$@"
python3 tools/pmc_traffic.py "$OUT"
