#!/bin/bash
# Ablations of the ordered mask-replay path on config 2's table (diagnostics
# library): 1 = no verify / replay, 2 = no probe, 4 = no replay adds, 32 = no argmax
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for a in ${ABL:-0 1 2 4 32}; do
  LDGPU_ABLATE=$a timeout -k 10 200 python3 -u bench.py --path replay --steps 10 --warmup 2 --no-cpu-baseline --no-host-path --no-alt-paths > gpurun_out/abl/r.log 2>&1 || { echo "fail $a"; tail -5 gpurun_out/abl/r.log; exit 1; }
  echo "replay ablate=$a $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abl/r.log)"
done
