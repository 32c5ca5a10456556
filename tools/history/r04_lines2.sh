#!/bin/bash
# Round-4 final lines: FIT (config 3 shard), config 4, config 5, FIT at the
# L = 200 shape with its kernel trace, and a FIT host-phase trace (diagnostics build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/lines2; mkdir -p $O
for c in "fit:--mode fit --steps 3 --warmup 1" "c4:--config 4" "c5:--config 5 --steps 5 --warmup 1"; do
  t=${c%%:*}; a=${c#*:}
  echo "== $t"
  timeout -k 10 600 python3 -u bench.py $a --json-out $O/$t.json > $O/$t.log 2>&1 || { tail -5 $O/$t.log; exit 1; }
  tail -c 200 $O/$t.log; echo
done
LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 300 python3 -u bench.py --mode fit --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/fit_trace.json > $O/fit_trace.log 2>&1 || { tail -5 $O/fit_trace.log; exit 1; }
tools/history/r04_prof.sh fitL200b "--mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 --steps 1 --warmup 0 --cpu-seconds 20" > /dev/null 2>&1 || exit 1
echo done
