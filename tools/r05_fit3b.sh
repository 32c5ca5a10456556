#!/bin/bash
# Round 5: config 3's count -- per-batch host phases (diagnostics trace) and
# the kernel trace of the product path (sum of kernel time vs count time).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_fit3b; mkdir -p $O
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 300 python3 -u bench.py --mode fit \
  --steps 2 --warmup 1 --no-cpu-baseline --count-only --json-out $O/trace.json > $O/trace.log 2>&1 || { tail -n 20 $O/trace.log; exit 1; }
grep "fit batch" $O/trace.log | tail -n 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py --mode fit --steps 2 \
  --warmup 1 --no-cpu-baseline --count-only --json-out $O/prof.json > $O/prof.log 2>&1 || { tail -n 20 $O/prof.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/prof.json'));print(d['phases_s'], d['count_s_per_step'])"
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/prof
