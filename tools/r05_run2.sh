#!/bin/bash
# Round 5: status agreement / JNI / bucket-layout / top-K tests, config 4
# (product, then the diagnostics library with LDGPU_BUCKETS=0 / 1 for a
# same-box A/B), the config-5-shaped fit with the host trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_run2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_distributed.py \
  tests/test_jni_shim.py tests/test_gpu_score.py tests/test_gpu_fit.py \
  -k "fail or jni or shim or chunk_layout or config4 or config5_timed or product_library or fit_table or config3 or 4096 or bench_fit or distributed" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -u bench.py --config 4 --no-host-path --json-out $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/c4.json'));print('c4 product', d['value'], d['ms_per_step'], d.get('labels_match_oracle'))"
for b in 0 1; do
  LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_BUCKETS=$b timeout -k 10 300 python3 -u bench.py --config 4 \
    --no-host-path --no-cpu-baseline --no-alt-paths --json-out $O/c4_b$b.json > $O/c4_b$b.log 2>&1 || { tail -20 $O/c4_b$b.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c4_b$b.json'));print('c4 diag buckets=$b', d['value'], d['ms_per_step'])"
done
LDGPU_LIB=$PWD/spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_TRACE=1 timeout -k 10 400 python3 -u bench.py \
  --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 --steps 1 --warmup 0 \
  --json-out $O/fit_L200.json > $O/fit_L200.log 2>&1 || { tail -30 $O/fit_L200.log; exit 1; }
grep -E "fit (table|v5 batch)" $O/fit_L200.log | head -14
python3 -c "import json;d=json.load(open('$O/fit_L200.json'));print(d['phases_s'],d.get('counts_match_oracle'))"
