#!/bin/bash
# Round 5: FIT v5 parity tests, then the config-5-shaped fit (L=200, grams
# 1-7, K=50k, 1 GB) on the diagnostics library with the host trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_fit; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fit.py \
  -k "count_paths or 4096 or counts_match or growth or single_language or config3" > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 400 python3 -u bench.py \
  --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 --steps 1 --warmup 0 \
  --json-out $O/fit_L200.json > $O/fit_L200.log 2>&1 || { tail -30 $O/fit_L200.log; exit 1; }
grep -E "fit v5|count_s|counts_match" $O/fit_L200.log | tail -20
python3 -c "import json;d=json.load(open('$O/fit_L200.json'));print(d['phases_s'],d.get('counts_match_oracle'))"
