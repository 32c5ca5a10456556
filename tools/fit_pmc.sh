#!/bin/bash
# HBM traffic of one FIT count from PMC counters (MI355X_MICROARCH.md HBM
# section): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (no
# tracing) over `bench.py --mode fit --steps 1 --warmup 0 --count-only` (two
# counts: the timed one and the statistics one, no top-K table), summed per
# kernel over the ldgpu kernels and the radix sorts (rocprim: FIT v5's; other
# rocprim kernels -- torch's, drawing the corpus -- apart), then
# tools/fit_pmc.py calibrates the raw counters on kernels whose bytes are
# known exactly (FIT v4: part2 reads and writes every record once; FIT v5:
# sort_emit writes one 8-B key per corpus byte, sort_runs reads the keys).
# Usage: tools/fit_pmc.sh <outdir> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== $ctr"
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex 'ldgpu|rocprim' --output-format csv -d "$PWD/$OUT/$ctr" -o run -- \
      python3 bench.py --mode fit --steps 1 --warmup 0 --no-cpu-baseline --count-only --json-out "$PWD/$OUT/$ctr.json" "$@" > "$OUT/$ctr.log" 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$ctr.log"; exit $rc; }
  f=$(find "$OUT/$ctr" -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$ctr" > "$OUT/$ctr.sum" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if r["Counter_Name"] != sys.argv[2]:
        continue
    if "rocprim" in k and "ldgpu" not in k:
        # the radix sorts (FIT v5's own); any other rocprim kernel (torch's
        # boolean indexing while the corpus is drawn) is kept apart
        k = "rocprim_radix_sort" if "radix_sort" in k else "rocprim_other"
    elif "ldgpu" in k:
        k = k.split("(ldgpu")[0].replace("ldgpu::(anonymous namespace)::", "").replace("void ", "")
    else:
        continue
    tot[k] += float(r["Counter_Value"]); n[k] += 1
for k in sorted(tot):
    print(f"{k}\t{n[k]}\t{tot[k]:.1f}")
PY
  rm -rf "$OUT/$ctr"
done
python3 tools/fit_pmc.py "$OUT"
