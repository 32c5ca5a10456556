"""Summarise tools/gather_cal.sh: FETCH_SIZE (and TCC request / hit counters)
of the known-byte stream and random-gather kernels of tools/gather_cal.hip
-> <out>/gather_cal.json (copy to profiles/ to keep it).

read_factor_stream  = known streamed bytes / FETCH_SIZE bytes
fetch_per_gather_B  = FETCH_SIZE bytes / random 4-B gathers
read_factor_gather  = (distinct 64-B lines x 64) / FETCH_SIZE bytes
"""
import csv
import glob
import json
import os
import sys


def last_values(d, kernel):
    """counter -> value of the kernel's last dispatch (the timed one)."""
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            did = int(row["Dispatch_Id"])
            per.setdefault(did, {}).setdefault(row["Counter_Name"], 0.0)
            per[did][row["Counter_Name"]] += float(row["Counter_Value"])
    return per[max(per)] if per else {}


def main(out):
    known = json.load(open(os.path.join(out, "plain.json")))
    res = {"known": known}
    for kern in ("stream_kernel", "gather_kernel"):
        vals = {}
        for d in sorted(glob.glob(os.path.join(out, "*"))):
            if os.path.isdir(d):
                vals.update(last_values(d, kern))
        res[kern] = vals
    fs = res["stream_kernel"].get("FETCH_SIZE")
    fg = res["gather_kernel"].get("FETCH_SIZE")
    if fs:
        res["read_factor_stream"] = round(known["stream_known_bytes"] / (fs * 1024.0), 4)
    if fg:
        res["fetch_per_gather_B"] = round(fg * 1024.0 / known["gather_loads"], 3)
        res["read_factor_gather"] = round(known["gather_distinct_lines_expected"] * 64.0 / (fg * 1024.0), 4)
    for kern in ("stream_kernel", "gather_kernel"):
        h, m = res[kern].get("TCC_HIT_sum"), res[kern].get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            res[kern + "_l2_hit_rate"] = round(h / (h + m), 4)
    res["note"] = ("FETCH_SIZE in KiB x 1024; gather = one random 4-B load per 64-B line of a buffer far beyond "
                   "the 256 MiB MALL; factors are known bytes / counter bytes")
    with open(os.path.join(out, "gather_cal.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
