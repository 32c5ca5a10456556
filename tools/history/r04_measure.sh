#!/bin/bash
# Round-4 measurement pass: FIT kernel trace (config 3 shard), config-4/5 PMC
# traffic, the config-5 and L=200 FIT bench lines with their kernel traces.
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/history/r04_prof.sh fit3 "--mode fit --steps 3 --warmup 1" || exit $?
tools/pmc_traffic.sh gpurun_out/pmc_c4 --config 4 --docs 25000000 > gpurun_out/pmc_c4.log 2>&1 || { tail -5 gpurun_out/pmc_c4.log; exit 1; }
tools/pmc_traffic.sh gpurun_out/pmc_c5 --config 5 --docs 2000000 > gpurun_out/pmc_c5.log 2>&1 || { tail -5 gpurun_out/pmc_c5.log; exit 1; }
rm -rf gpurun_out/pmc_c4/*_real gpurun_out/pmc_c4/*_cal gpurun_out/pmc_c5/*_real gpurun_out/pmc_c5/*_cal
tools/history/r04_prof.sh fitL200 "--mode fit --langs 200 --grams 1,2,3,4,5,6,7 --profile-size 50000 --fit-bytes 1000000000 --steps 1 --warmup 0 --cpu-seconds 20" || exit $?
