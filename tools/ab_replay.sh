#!/bin/bash
# A/B of diagnostics builds on the ordered mask-replay path (config 2's table):
#   LIBS="d0 d1" ROUNDS=2 tools/ab_replay.sh   (lib X = lib/libldgpu_X.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abr
for r in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-d0 d1}; do
    LDGPU_DIAG_LIB=spark-languagedetector_amd/lib/libldgpu_$lib.so timeout -k 10 200 python3 -u bench.py --path replay --steps 20 --warmup 3 \
        --no-cpu-baseline --no-host-path --no-alt-paths > gpurun_out/abr/x.log 2>&1 || { echo "fail $lib"; tail -5 gpurun_out/abr/x.log; exit 1; }
    echo "replay lib=$lib $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abr/x.log)"
  done
done
if [ -n "${CHECK:-}" ]; then
  LDGPU_DIAG_LIB=spark-languagedetector_amd/lib/libldgpu_$CHECK.so timeout -k 10 300 python3 -u bench.py --path replay --steps 5 --warmup 1 \
      --no-host-path --no-alt-paths --json-out gpurun_out/abr/check.json > gpurun_out/abr/check.log 2>&1 || { tail -5 gpurun_out/abr/check.log; exit 1; }
  echo "check $CHECK $(grep -o '"labels_match_oracle": [a-z]*' gpurun_out/abr/check.json | head -1)"
fi
