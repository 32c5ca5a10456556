#!/bin/bash
# Round 5: config 5 -- A/B of the cold-parameter keyed kernels, then the SQ
# counters of the product kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIBS="c5base c5cold" CFGS="--config 5" ROUNDS=2 STEPS=5 tools/ab.sh || exit 1
O=gpurun_out/r05_c5; mkdir -p $O
ONLY="1 2 3" tools/pmc_profile.sh $O/sq_c5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths \
  > $O/sq_c5.log 2>&1 || { tail -20 $O/sq_c5.log; exit 1; }
grep -A30 "score_kernel" $O/sq_c5/summary.txt | head -40
