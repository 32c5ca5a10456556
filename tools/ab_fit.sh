#!/bin/bash
# Same-box A/B of FIT lines for library builds: LIBS="A B" ROUNDS=2 tools/ab_fit.sh [bench fit args...]
# (library X = spark-languagedetector_amd/lib/libldgpu_X.so, B = libldgpu.so); prints count / table ms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-A B}; do
    f=spark-languagedetector_amd/lib/libldgpu_$lib.so; [ "$lib" = B ] && f=spark-languagedetector_amd/lib/libldgpu.so
    LDGPU_LIB=$f timeout -k 10 400 python3 -u bench.py --mode fit "$@" --no-cpu-baseline --json-out gpurun_out/ab/fit_$lib.json > gpurun_out/ab/fit_$lib.log 2>&1 \
      || { echo "fail $lib"; tail -5 gpurun_out/ab/fit_$lib.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/fit_$lib.json'));r=d['roofline'];print('lib=$lib', 'count_ms', r['count_ms'], 'phases', d['phases_s'], 'match', d.get('counts_match_oracle'))"
  done
done
