#!/bin/bash
# Round 5: general-key SCORE path after staging documents in LDS -- its parity
# tests, then config 2's line (general_keys_path side measurement).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_gen; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_score.py tests/test_gpu_fit.py \
  -k "long or general or wide" > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 3 --no-host-path --json-out $O/bench_config2.json > $O/bench.log 2>&1 \
  || { tail -n 30 $O/bench.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_config2.json'));print(d['value'], d['ms_per_step']);print(json.dumps(d.get('general_keys_path')))"
