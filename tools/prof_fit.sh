#!/bin/bash
# rocprofv3 kernel-trace stats of the fit bench.  Usage: tools/prof_fit.sh tag [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-proffit}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 -u bench.py --mode fit --steps 1 --warmup 1 --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
rc=$?; tail -c 1500 "$OUT/bench.log"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; 2>/dev/null
rm -rf "$OUT/prof"   # the full trace (>64 MiB with the corpus generator's kernels) stays on the box
cut -d, -f1-8 "$OUT/kernel_stats.csv" 2>/dev/null | head -20
exit $rc
