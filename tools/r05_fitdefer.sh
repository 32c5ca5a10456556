#!/bin/bash
# Round 5: FIT parity after deferring each batch's last merge readback, then
# config 3's fit line (product) and its per-batch host phases (diagnostics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_fitdefer; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fit.py tests/test_distributed.py \
  -m gpu > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 400 python3 -u bench.py --mode fit --steps 5 --warmup 1 --json-out $O/bench_fit.json > $O/bench_fit.log 2>&1 \
  || { tail -n 20 $O/bench_fit.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_fit.json'));print(d['value'], d['count_ms_per_gib'], d['phases_s'], d.get('counts_match_oracle'))"
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 300 python3 -u bench.py --mode fit \
  --steps 1 --warmup 1 --no-cpu-baseline --count-only > $O/trace.log 2>&1 || { tail -n 20 $O/trace.log; exit 1; }
grep "fit batch" $O/trace.log | tail -n 4
