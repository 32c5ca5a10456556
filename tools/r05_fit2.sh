#!/bin/bash
# Round 5: config-5-shaped fit with the host trace (diagnostics library,
# warmup + step: three counts on one context), then its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_fit2; mkdir -p $O
A="--mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000"
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 400 python3 -u bench.py \
  $A --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/fit_L200_trace.json > $O/fit_L200_trace.log 2>&1 || { tail -30 $O/fit_L200_trace.log; exit 1; }
grep -E "fit (grow|table|v5 batch)|count " $O/fit_L200_trace.log | tail -60
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o fit -- python3 -u bench.py $A --steps 1 --warmup 0 \
  --no-cpu-baseline --json-out $O/fit_L200_prof.json > $O/fit_L200_prof.log 2>&1 || { tail -30 $O/fit_L200_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/fit_L200_kernel_stats.csv
python3 tools/kstats.py $O/fit_L200_kernel_stats.csv 2>/dev/null | head -30 || head -c 3000 $O/fit_L200_kernel_stats.csv
rm -rf $O/prof
