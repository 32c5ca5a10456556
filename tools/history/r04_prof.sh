#!/bin/bash
# Kernel-trace profile of one bench run: rocprofv3 --kernel-trace --stats,
# the kernel stats CSV copied to gpurun_out/TAG/kernel_stats.csv.
#   tools/history/r04_prof.sh TAG "bench args"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; ARGS=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 -u bench.py $ARGS --json-out "$OUT/bench.json" > "$OUT/log" 2>&1
rc=$?
tail -c 600 "$OUT/log"; echo
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && python3 tools/kstats.py "$OUT/kernel_stats.csv" | head -n 30
rm -rf "$OUT/prof"   # the per-dispatch trace: too large to copy back
exit $rc
