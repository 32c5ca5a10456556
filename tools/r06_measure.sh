#!/bin/bash
# Round 6 measurement at HEAD for one workload: PMC traffic (FETCH / WRITE
# passes + empty-table calibration + L2), SQ counters, then the bench line
# (which reads the PMC file just written) and the rocprofv3 kernel-trace stats.
# Usage: tools/r06_measure.sh <name> <pmc-json-name> <sq-docs> [bench args...]
#   e.g. tools/r06_measure.sh c4 pmc_traffic_config4.json 25000000 --config 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=$1; PMC=$2; SQDOCS=$3; shift 3
OUT=gpurun_out/r06m_$NAME; mkdir -p $OUT
echo "== pmc traffic $NAME"
tools/pmc_traffic.sh $OUT/pmc "$@" > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
cp $OUT/pmc/pmc_traffic.json profiles/$PMC && cp $OUT/pmc/pmc_traffic.json $OUT/$PMC
rm -rf $OUT/pmc/fetch_* $OUT/pmc/write_* $OUT/pmc/l2_real
echo "== sq counters $NAME"
ONLY="1 2 3" tools/pmc_profile.sh $OUT/sq "$@" --docs $SQDOCS --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
cp $OUT/sq/summary.txt $OUT/sq_summary.txt; rm -rf $OUT/sq/pass*
echo "== bench $NAME"
timeout -k 10 600 python -u bench.py "$@" ${BENCH_EXTRA:-} --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -c 600 $OUT/bench.json
echo "== rocprof $NAME"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run \
  -- python3 bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
head -5 $OUT/kernel_stats.csv | cut -c1-150
echo "== done $NAME"
