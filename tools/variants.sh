#!/bin/bash
# Time the SCORE kernel under several library builds / env settings.
# usage: tools/variants.sh OUTTAG "name|ENV=.. ENV2=.." ...   (bench args via BENCH_ARGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%|*}; envs=${spec#*|}
  env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path ${BENCH_ARGS:-} > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -o '"kernel_ms": [0-9.]*' "$OUT/$name.log")"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
done
