#!/bin/bash
# Round 5: FIT v5 parity after batching runs_add's probes, then the
# config-5-shaped fit line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_runs; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fit.py \
  -k "count_paths or config5_shape or config3_shape or growth or 4096 or sparse or two_count" > $O/tests.log 2>&1 \
  || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 500 python3 -u bench.py --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 \
  --steps 2 --warmup 1 --json-out $O/bench_fit_L200.json > $O/bench_fit_L200.log 2>&1 || { tail -n 20 $O/bench_fit_L200.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_fit_L200.json'));print('L200', d['value'], d['phases_s'], d.get('counts_match_oracle'))"
