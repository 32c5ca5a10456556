#!/bin/bash
# Round 6 FIT measurement at HEAD: PMC traffic of the count (tools/fit_pmc.sh,
# count-only run), then the bench line (reads the PMC file just written) and
# the rocprofv3 kernel-trace stats.
# Usage: tools/r06_measure_fit.sh <name> <pmc-json-name> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=$1; PMC=$2; shift 2
OUT=gpurun_out/r06m_$NAME; mkdir -p $OUT
if [ -z "${SKIP_PMC:-}" ]; then
  echo "== fit pmc $NAME"
  tools/fit_pmc.sh $OUT/pmc "$@" > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
  cp $OUT/pmc/pmc_traffic_fit.json profiles/$PMC && cp $OUT/pmc/pmc_traffic_fit.json $OUT/$PMC
fi
echo "== bench $NAME"
timeout -k 10 900 python -u bench.py --mode fit "$@" ${BENCH_EXTRA:-} --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -c 800 $OUT/bench.json
echo "== rocprof $NAME"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run \
  -- python3 bench.py --mode fit "$@" --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
grep ldgpu $OUT/kernel_stats.csv | head -12 | cut -c1-160
echo "== done $NAME"
