#!/bin/bash
# rocprofv3 kernel-trace stats of score benches (score kernels only, the
# summary kept): tools/prof_score.sh <tag> "<bench args>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
i=0
for a in "$@"; do
  i=$((i+1))
  OUT=gpurun_out/$TAG/p$i
  mkdir -p "$OUT"
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 -u bench.py --no-cpu-baseline --no-host-path --no-alt-paths --json-out "$PWD/$OUT/bench.json" $a > "$OUT/bench.log" 2>&1
  rc=$?; echo "== $a rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.log"; exit $rc; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
  rm -rf "$OUT/prof"
  grep -E "score_kernel|combine" "$OUT/kernel_stats.csv" | cut -d, -f1-4 | sed 's/(ldgpu[^"]*//'
done
