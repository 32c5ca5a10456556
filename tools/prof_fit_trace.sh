#!/bin/bash
# rocprofv3 kernel trace of one fit count (bench --mode fit --steps 1 --warmup 0):
# the ldgpu kernels in launch order with their durations (the full trace, with
# the corpus generator's kernels, stays on the box).  Usage: tools/prof_fit_trace.sh tag [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prof_trace}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 -u bench.py --mode fit --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
rc=$?; tail -c 600 "$OUT/bench.log"
f=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python3 - "$f" > "$OUT/ldgpu_trace.txt" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ldgpu" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows:
    n = r["Kernel_Name"].split("(ldgpu")[0].replace("ldgpu::(anonymous namespace)::", "").replace("void ", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:10.3f} ms  {(e - s) / 1e6:8.3f} ms  {n}")
PY
rm -rf "$OUT/prof"
head -c 400 "$OUT/ldgpu_trace.txt"
exit $rc
