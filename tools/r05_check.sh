#!/bin/bash
# Round 5: score parity after the keyed preload (keyed layouts, config 4/5
# shapes), the config-5 bench line (product library, oracle-checked sample),
# the L200 fit (table phase), then diagnostics ablations of configs 4 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_check; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_score.py \
  -k "keyed or config4 or config5 or bucket or chunk or line" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u bench.py --config 5 --steps 5 --warmup 1 --no-host-path --json-out $O/c5.json > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['value'], d['ms_per_step'], d.get('labels_match_oracle'), d.get('oracle_check'))"
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 400 python3 -u bench.py \
  --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 --steps 1 --warmup 0 --no-cpu-baseline \
  --json-out $O/fit_L200.json > $O/fit_L200.log 2>&1 || { tail -30 $O/fit_L200.log; exit 1; }
grep -E "fit table" $O/fit_L200.log | head -14
python3 -c "import json;d=json.load(open('$O/fit_L200.json'));print(d['phases_s'])"
for cfg in "--config 4" "--config 5 --steps 5"; do
for a in 0 1 2 8 16 32; do
  LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_ABLATE=$a timeout -k 10 300 python3 -u bench.py $cfg --warmup 2 \
    --no-cpu-baseline --no-host-path --no-alt-paths > $O/abl.log 2>&1 || { echo "fail $cfg $a"; tail -5 $O/abl.log; exit 1; }
  echo "$cfg ablate=$a $(grep -o '"kernel_ms": [0-9.]*' $O/abl.log)"
done
done
