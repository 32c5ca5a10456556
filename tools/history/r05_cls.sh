#!/bin/bash
# Round 5: class mode -- its parity tests and the replay-path tests, then
# config 2's bench line (mask_replay_path: class mode / ordered / two values).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_cls; mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_classes.py \
  "tests/test_gpu_score.py::test_random_parity" "tests/test_gpu_score.py::test_uniform_value_parity" \
  "tests/test_gpu_score.py::test_fast_path_queue_flush_mid_document" > $O/tests.log 2>&1 \
  || { tail -n 40 $O/tests.log; exit 1; }
tail -n 3 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --json-out $O/bench_config2.json > $O/bench.log 2>&1 \
  || { tail -n 30 $O/bench.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r05_cls/bench_config2.json"))
print(d["value"], d["ms_per_step"], d["labels_match_oracle"])
print(json.dumps(d["mask_replay_path"], indent=1))
PY
