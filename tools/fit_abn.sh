#!/bin/bash
# FIT A/B of library builds on ONE box (config 3's shard unless BYTES is set):
#   LIBS="f0 f1" ROUNDS=2 tools/fit_abn.sh   (lib X = lib/libldgpu_X.so, B = libldgpu.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fab
export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-A B}; do
    f=spark-languagedetector_amd/lib/libldgpu_$lib.so; [ "$lib" = B ] && f=spark-languagedetector_amd/lib/libldgpu.so
    LDGPU_LIB=$f timeout -k 10 300 python3 -u bench.py --mode fit --fit-bytes ${BYTES:-6250000000} --steps ${STEPS:-3} --warmup 1 \
        --no-cpu-baseline ${FITARGS:-} --json-out gpurun_out/fab/$lib.json > gpurun_out/fab/x.log 2>&1 \
      || { echo "fail $lib"; tail -5 gpurun_out/fab/x.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/fab/$lib.json'));print('lib=$lib', d['count_ms_per_gib'], d['phases_s']['count_s'], d['phases_s']['table_s'], d['windows_counted_exactly_once'])"
  done
done
