#!/bin/bash
# One GPU-box pass: gpu tests -> smoke -> bench -> rocprofv3 kernel-trace stats.
# Stops at the first step that faults / aborts / times out (anything but a
# plain test failure, rc 1).  Usage: tools/gpu_check.sh [tag] [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py "$@"
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-path
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; 2>/dev/null
echo "== done"; cat "$OUT/kernel_stats.csv" 2>/dev/null | head -20
