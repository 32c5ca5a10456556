#!/bin/bash
# One rocprofv3 SQ-counter pass per library variant over a short bench run.
# Usage: tools/pmc_compare.sh OUTTAG "name|ENV=.." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
CTR=${CTR:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT"}
for spec in "$@"; do
  name=${spec%%|*}; envs=${spec#*|}
  for e in $envs; do export "$e"; done
  timeout -s KILL 240 rocprofv3 --pmc $CTR --output-format csv -d "$PWD/$OUT/$name/pass1" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --docs 4000000 > "$OUT/$name.log" 2>&1
  rc=$?
  for e in $envs; do unset "${e%%=*}"; done
  echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
  python3 tools/pmc_summary.py "$OUT/$name" | grep -A20 score_kernel | head -12
done
