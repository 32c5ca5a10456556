#!/bin/bash
# Round 6: FIT parity tests, then A/B of the FIT v5 count at config 5's fit
# shape (L = 200, grams 1-7, 1 GB) and of FIT v4 at config 3 (1 GB): LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06fit; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fit.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
  rc=$?; tail -n 2 $OUT/t.log; grep -E "FAILED|Error" $OUT/t.log | head; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for lib in ${LIBS:-fitbase B}; do
    f=spark-languagedetector_amd/lib/libldgpu_$lib.so; [ "$lib" = B ] && f=spark-languagedetector_amd/lib/libldgpu.so
    LDGPU_LIB=$PWD/$f timeout -k 10 300 python3 -u bench.py --mode fit --langs 200 --grams 1,2,3,4,5,6,7 \
      --profile-size 50000 --fit-bytes 1000000000 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/l200_$lib.json 2> $OUT/l200_$lib.err \
      || { echo "fail $lib"; tail -5 $OUT/l200_$lib.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],'L200 count_s',d['count_s_per_step'],'table_s',d['phases_s']['table_s'])" $OUT/l200_$lib.json $lib
    LDGPU_LIB=$PWD/$f timeout -k 10 300 python3 -u bench.py --mode fit --fit-bytes 1073741824 --steps 2 --warmup 1 \
      --no-cpu-baseline > $OUT/c3_$lib.json 2> $OUT/c3_$lib.err || { echo "fail c3 $lib"; tail -5 $OUT/c3_$lib.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],'c3 1GiB count ms/GiB',d['count_ms_per_gib'])" $OUT/c3_$lib.json $lib
  done
done
