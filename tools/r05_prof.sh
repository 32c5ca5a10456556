#!/bin/bash
# Round 5 profiles: the config-5-shaped fit (FIT v5) -- PMC traffic of the
# count and a kernel trace of the whole fit -- and config 4's SQ counters and
# traffic with the bucket key table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_prof; mkdir -p $O
A="--langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000"
tools/fit_pmc.sh $O/pmc_fit_L200 $A > $O/pmc_fit_L200.log 2>&1 || { tail -20 $O/pmc_fit_L200.log; exit 1; }
python3 tools/fit_pmc.py $O/pmc_fit_L200 pmc_traffic_fit_L200.json | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/trace -o fit -- python3 -u bench.py \
  --mode fit $A --steps 1 --warmup 0 --no-cpu-baseline --json-out $O/fit_trace.json > $O/fit_trace.log 2>&1 || { tail -20 $O/fit_trace.log; exit 1; }
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp "$f" $O/fit_L200_kernel_stats.csv; rm -rf $O/trace
python3 tools/kstats.py $O/fit_L200_kernel_stats.csv . | head -24
ONLY="1 2 3" tools/pmc_profile.sh $O/sq_c4 --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths \
  > $O/sq_c4.log 2>&1 || { tail -20 $O/sq_c4.log; exit 1; }
grep -A40 "score_kernel" $O/sq_c4/summary.txt | head -60
tools/pmc_traffic.sh $O/tr_c4 --config 4 > $O/tr_c4.log 2>&1 || { tail -20 $O/tr_c4.log; exit 1; }
tail -5 $O/tr_c4.log
