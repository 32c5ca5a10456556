#!/bin/bash
# Round 5: FIT parity (all of test_gpu_fit + persistence) after the pinned
# table cache, then the config-5-shaped fit line with its phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_fit3; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fit.py tests/test_persistence.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 400 python3 -u bench.py \
  --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 --steps 1 --warmup 0 --no-cpu-baseline \
  --json-out $O/fit_L200_diag.json > $O/fit_L200_diag.log 2>&1 || { tail -30 $O/fit_L200_diag.log; exit 1; }
grep -E "fit table" $O/fit_L200_diag.log | head -14
timeout -k 10 400 python3 -u bench.py --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 \
  --steps 2 --warmup 1 --json-out $O/fit_L200.json > $O/fit_L200.log 2>&1 || { tail -30 $O/fit_L200.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/fit_L200.json'));print(d['phases_s'], d['value'], d.get('counts_match_oracle'), d['roofline'])"
