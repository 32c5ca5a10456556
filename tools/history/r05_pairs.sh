#!/bin/bash
# Round 5: FIT parity with T's pair table interleaved, then the
# config-5-shaped fit line (L = 200, grams 1-7, 1 GB) and config 3's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_pairs; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fit.py tests/test_distributed.py \
  tests/test_persistence.py -m gpu > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 500 python3 -u bench.py --mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 \
  --steps 2 --warmup 1 --json-out $O/bench_fit_L200.json > $O/bench_fit_L200.log 2>&1 || { tail -n 20 $O/bench_fit_L200.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_fit_L200.json'));print('L200', d['value'], d['phases_s'], d.get('counts_match_oracle'))"
timeout -k 10 400 python3 -u bench.py --mode fit --steps 5 --warmup 1 --json-out $O/bench_fit.json > $O/bench_fit.log 2>&1 \
  || { tail -n 20 $O/bench_fit.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_fit.json'));print('c3', d['value'], d['count_ms_per_gib'], d['phases_s'], d.get('counts_match_oracle'))"
