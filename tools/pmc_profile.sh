#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, never combined with tracing)
# over a short bench run; summaries by tools/pmc_summary.py.
# Usage: tools/pmc_profile.sh <outdir> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for pass in "${PASSES[@]}"; do
  i=$((i+1))
  if [ -n "${ONLY:-}" ] && [[ " $ONLY " != *" $i "* ]]; then continue; fi
  echo "== pass $i: $pass"
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$PWD/$OUT/pass$i" -o run -- python3 bench.py "$@" > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/summary.txt"
