#!/bin/bash
# Round 6: config 4 -- A/B of the pack kernel's sub-block-outer probe
# (LDGPU_PACK_KOUTER) against the all-sub-blocks probe, then WRITE_SIZE of
# each (PMC pass, 25M documents).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06c4; mkdir -p $OUT
[ -n "${SKIP_AB:-}" ] || LIBS="${LIBS:-n4base n4k}" CFGS="--config 4" ROUNDS=${ROUNDS:-2} STEPS=10 tools/ab.sh || exit 1
for lib in ${LIBS:-n4base n4k}; do
  LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_$lib.so timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE \
    --kernel-include-regex score_kernel --output-format csv -d $PWD/$OUT/w_$lib -o run -- python3 bench.py --config 4 \
    --docs 25000000 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths > $OUT/w_$lib.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $lib rc=$rc"; tail -5 $OUT/w_$lib.log; exit $rc; }
  f=$(find $OUT/w_$lib -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys, collections
t = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    t[r["Kernel_Name"][:48]] += float(r["Counter_Value"]); n[r["Kernel_Name"][:48]] += 1
for k in t: print(sys.argv[2], k, "launches", n[k], "WRITE_SIZE KB per launch", round(t[k] / n[k]))
PY
done
