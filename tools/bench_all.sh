#!/bin/bash
# Bench pass on one GPU box: config 2 headline (full line: cpu_baseline,
# oracle label check, host path), its rocprofv3 kernel-trace stats, then
# configs 4 / 5 and the config-3 FIT line.  Each step has its own time limit;
# the first step that fails ends the script.  Usage: tools/bench_all.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -c 1500 "$OUT/$name.log"; echo
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
ONLY=${ONLY:-c2 prof c4 c5 fit}
for s in $ONLY; do
  case $s in
    c2)   step bench_c2 300 python -u bench.py --json-out "$OUT/bench_c2.json" ;;
    prof) step rocprof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_c2" -o run \
            -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths
          find "$OUT/prof_c2" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_c2.csv" \; ;;
    c4)   step bench_c4 400 python -u bench.py --config 4 --steps 10 --warmup 2 --json-out "$OUT/bench_c4.json" ;;
    c5)   step bench_c5 500 python -u bench.py --config 5 --steps 5 --warmup 1 --no-host-path --json-out "$OUT/bench_c5.json" ;;
    fit)  step bench_fit 400 python -u bench.py --mode fit --steps 5 --warmup 1 --json-out "$OUT/bench_fit.json" ;;
  esac
done
echo "== done"
