#!/bin/bash
# Round 5: the config-5-shaped fit parity test, then config 2's bench line
# (with the general-key and static-detect side paths).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_fit5; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread \
  "tests/test_gpu_fit.py::test_config5_shape_fit_counts_table_and_scores" > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 3 --json-out $O/bench_config2.json > $O/bench_config2.log 2>&1 \
  || { tail -n 30 $O/bench_config2.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_config2.json'));print(d['value'], d['ms_per_step'], d.get('oracle_check'));print(json.dumps(d.get('general_keys_path')))"
