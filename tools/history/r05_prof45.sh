#!/bin/bash
# Round 5: rocprofv3 kernel-trace stats of configs 4 and 5 (product library),
# the same commands as their bench lines minus the CPU legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_prof45; mkdir -p $O
for c in 4 5; do
  st=10; [ $c = 5 ] && st=5
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/p$c -o run -- python3 bench.py --config $c \
    --steps $st --warmup 1 --no-cpu-baseline --no-host-path --no-alt-paths --json-out $O/bench_c$c.json > $O/prof_c$c.log 2>&1 \
    || { tail -n 20 $O/prof_c$c.log; exit 1; }
  find $O/p$c -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c$c.csv \;
  rm -rf $O/p$c
  python3 -c "import json;d=json.load(open('$O/bench_c$c.json'));print($c, d['ms_per_step'], d['roofline']['kernel_ms'])"
done
