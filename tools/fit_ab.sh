#!/bin/bash
# FIT A/B on the same untiled corpus: the round-2 library (lib/libldgpu_r02.so,
# built from git 554a7db) against the current one, then a kernel trace of the
# current one.  Usage: tools/fit_ab.sh TAG [fit bytes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; BYTES=${2:-1073741824}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/prof"
export TMPDIR=/tmp
ROOT=$PWD
A="--mode fit --fit-bytes $BYTES --steps 3 --warmup 1 --no-cpu-baseline"
echo "== r02 library"
LDGPU_LIB=$ROOT/spark-languagedetector_amd/lib/libldgpu_r02.so timeout -k 10 300 python -u bench.py $A --json-out $OUT/ab_r02.json > $OUT/ab_r02.log 2>&1 || { tail -5 $OUT/ab_r02.log; exit 1; }
python -c "import json;d=json.load(open('$OUT/ab_r02.json'));print('r02', d['count_ms_per_gib'], d['phases_s'])"
echo "== current library"
timeout -k 10 300 python -u bench.py $A --json-out $OUT/ab_cur.json > $OUT/ab_cur.log 2>&1 || { tail -5 $OUT/ab_cur.log; exit 1; }
python -c "import json;d=json.load(open('$OUT/ab_cur.json'));print('cur', d['count_ms_per_gib'], d['phases_s'])"
echo "== trace"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o fit -- python3 $ROOT/bench.py --mode fit --fit-bytes $BYTES --steps 2 --warmup 0 --no-cpu-baseline > $ROOT/$OUT/trace.log 2>&1 || { tail -5 $ROOT/$OUT/trace.log; exit 1; }
f=$(find $ROOT/$OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $ROOT/$OUT/kernel_stats.csv
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$ROOT/$OUT/kernel_stats.csv")))
for r in rows[:14]: print(round(float(r["TotalDurationNs"])/1e6,2), r["Calls"], r["Name"][:90])
PY
