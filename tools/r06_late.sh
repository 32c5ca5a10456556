#!/bin/bash
# Round 6: A/B of the late next-group offsets load (LDGPU_LATE_OFFSETS) on
# configs 4 and 5 (narrow builds), WRITE_SIZE of config 4's kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIBS="n4k n4late" CFGS="--config 4" ROUNDS=2 STEPS=10 tools/ab.sh || exit 1
SKIP_AB=1 LIBS="n4late" tools/r06_c4.sh 2>&1 | grep WRITE_SIZE
LIBS="n5base n5late" CFGS="--config 5" ROUNDS=2 STEPS=5 tools/ab.sh || exit 1
