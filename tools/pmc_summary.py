"""Summarise rocprofv3 --pmc CSV passes: per kernel, the mean per dispatch of
every counter (tools/pmc_profile.sh)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main(out):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(out, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")
                acc[k][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
    for k, cs in acc.items():
        if not re.search(os.environ.get("KERNELS", "score_kernel|count_kernel|emit_kernel|part2_kernel|reduce_kernel|merge_kernel"), k):
            continue
        print(k[:100])
        for c, vals in sorted(cs.items()):
            per = defaultdict(float)
            for d, v in vals:
                per[d] += v
            xs = list(per.values())
            print(f"  {c:32s} mean/dispatch {sum(xs) / len(xs):16.1f}   dispatches {len(xs)}")


if __name__ == "__main__":
    main(sys.argv[1])
