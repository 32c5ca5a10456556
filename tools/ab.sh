#!/bin/bash
# A/B timing of library builds on ONE box: for each config, each library in
# turn, ROUNDS times.  Usage: LIBS="A B C" CFGS="--config 2;..." tools/ab.sh
# (library X = spark-languagedetector_amd/lib/libldgpu_X.so, B = libldgpu.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
IFS=";" read -ra CF <<< "${CFGS:---config 2}"
for cfg in "${CF[@]}"; do
  for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-A B}; do
      f=spark-languagedetector_amd/lib/libldgpu_$lib.so; [ "$lib" = B ] && f=spark-languagedetector_amd/lib/libldgpu.so
      LDGPU_LIB=$f timeout -k 10 200 python3 -u bench.py $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-host-path --no-alt-paths > gpurun_out/ab/x.log 2>&1 \
        || { echo "fail $lib $cfg"; tail -5 gpurun_out/ab/x.log; exit 1; }
      echo "$cfg lib=$lib $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab/x.log) $(grep -o '"label_accuracy_vs_generator": [0-9.]*' gpurun_out/ab/x.log)"
    done
  done
done
