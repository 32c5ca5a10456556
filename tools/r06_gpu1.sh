#!/bin/bash
# Round 6: preprocess + score GPU tests, then the config-4 pack A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g1
timeout -k 10 600 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_score.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r06g1/t.log 2>&1
rc=$?; tail -3 gpurun_out/r06g1/t.log; grep -E "FAILED|Error" gpurun_out/r06g1/t.log | head; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
tools/r06_c4.sh
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r06g1/bench.json 2> gpurun_out/r06g1/bench.err
echo "bench rc=$?"; tail -c 1500 gpurun_out/r06g1/bench.json
