#!/bin/bash
# Per-dispatch durations of the library's kernels (and rocprim's), in launch
# order: tools/ktrace_seq.sh OUT bench-args...  -> OUT/seq.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 bench.py "$@" > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/seq.txt <<'PY'
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    n = r["Kernel_Name"]
    if "ldgpu" not in n and "rocprim" not in n:
        continue
    m = re.search(r"::(\w+)(<[^(]*>)?\(", n.replace("(anonymous namespace)", "anon"))
    name = m.group(1) if m else n[:40]
    if "rocprim" in n:
        name = "rocprim_" + (re.search(r"detail::(\w+)", n).group(1) if re.search(r"detail::(\w+)", n) else "?")
    print("%10.3f %s" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, name))
PY
rm -rf $OUT/prof
