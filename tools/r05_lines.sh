#!/bin/bash
# Round 5: pack-path parity, then the bench lines of configs 2 and 4
# (product library, oracle-checked samples, side paths).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_lines; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_score.py tests/test_gpu_classes.py \
  -k "pack or config4 or classes or class_mode or values" > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
for c in ${CFGS:-2 4}; do
  timeout -k 10 600 python3 -u bench.py --config $c --steps ${STEPS:-20} --warmup 3 --json-out $O/bench_config$c.json > $O/bench_config$c.log 2>&1 \
    || { tail -n 30 $O/bench_config$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_config$c.json'));print($c, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('oracle_check'));print(json.dumps(d.get('general_keys_path')))"
done
