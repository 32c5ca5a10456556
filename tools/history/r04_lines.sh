#!/bin/bash
# Round-4 bench lines: FIT PMC traffic refreshed first (profiles/ is read by
# bench.py for the counters' fields), then the FIT, config 4, 5 and 2 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/lines; mkdir -p $O
tools/fit_pmc.sh gpurun_out/pmc_fit > $O/pmc_fit.log 2>&1 || { tail -5 $O/pmc_fit.log; exit 1; }
cp gpurun_out/pmc_fit/pmc_traffic_fit.json profiles/pmc_traffic_fit.json
for c in "fit:--mode fit --steps 3 --warmup 1" "c4:--config 4" "c5:--config 5 --steps 5 --warmup 1" "c2:"; do
  t=${c%%:*}; a=${c#*:}
  echo "== $t"
  timeout -k 10 600 python3 -u bench.py $a --json-out $O/$t.json > $O/$t.log 2>&1 || { tail -5 $O/$t.log; exit 1; }
  tail -c 300 $O/$t.log; echo
done
