#!/bin/bash
# Round 5: A/B of narrow tuning builds on config 2 (LIBS), then one oracle-
# checked line of the last library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export LIBS="${LIBS:-n1base B}" CFGS="${CFGS:---config 2}"
ROUNDS=${ROUNDS:-3} STEPS=20 tools/ab.sh || exit 1
last=${LIBS##* }
lib=$PWD/spark-languagedetector_amd/lib/libldgpu_$last.so; [ "$last" = B ] && lib=$PWD/spark-languagedetector_amd/lib/libldgpu.so
LDGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py ${CFGS%%;*} --steps 5 --warmup 1 \
  --no-host-path --no-alt-paths --json-out gpurun_out/ab/check.json > gpurun_out/ab/check.log 2>&1 || { tail -n 20 gpurun_out/ab/check.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab/check.json'));print('check', d['ms_per_step'], d.get('oracle_check'))"
