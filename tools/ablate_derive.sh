#!/bin/bash
# Derive time attribution (diagnostics library): one fit count per setting of
# LDGPU_FIT_DERIVE_ABLATE = 0 (full), 1 (no adds to T), 2 (no prefix adds to
# T1), 3 (neither), kernel trace in launch order (tools/prof_fit_trace.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for a in ${ABLATE_SET:-0 1 2 3}; do
  LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_FIT_DERIVE_ABLATE=$a bash tools/prof_fit_trace.sh "${1:-abld}_a$a" "${@:2}" > /dev/null 2>&1 || { echo "ablate $a failed"; exit 1; }
  echo "ablate=$a"; awk '{s[$5]+=$3; c[$5]++} END {for (k in s) if (s[k] > 1) print "  ", k, c[k], s[k]}' "gpurun_out/${1:-abld}_a$a/ldgpu_trace.txt"
done
