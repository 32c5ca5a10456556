#!/bin/bash
# Quick perf check (no tests): config 2 and a 25M-document config 4 run,
# kernel times only.  Usage: tools/perf_quick.sh [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pq
export TMPDIR=/tmp
IFS=";" read -ra CFGS <<< "${PQ_CFGS:---config 2;--config 4 --docs 25000000}"
for cfg in "${CFGS[@]}"; do
  timeout -k 10 200 python3 -u bench.py $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-alt-paths "$@" > gpurun_out/pq/x.log 2>&1 \
    || { echo "fail $cfg"; tail -5 gpurun_out/pq/x.log; exit 1; }
  echo "$cfg $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/pq/x.log) $(grep -o '"label_accuracy_vs_generator": [0-9.]*' gpurun_out/pq/x.log)"
done
