"""Per-launch HBM traffic of score_kernel from tools/pmc_traffic.sh passes.

FETCH_SIZE / WRITE_SIZE are KiB (rocprofv3 derived counters).  The gfx950
correction is calibrated in this kernel's own access pattern: the empty-table
run reads exactly the document bytes + int64 offsets and writes the int32
labels, so  factor = known bytes / counter bytes  of that run, applied to the
real run (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of wide streaming
reads; other widths must be calibrated).
"""
import csv
import glob
import json
import os
import sys


def kernel_values(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "score_kernel" in row.get("Kernel_Name", "") and row["Counter_Name"] == counter:
                vals.setdefault(row["Dispatch_Id"], 0.0)
                vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    xs = [vals[k] for k in sorted(vals, key=lambda x: int(x))]
    return xs


def main(out):
    res = {}
    for name, ctr in (("fetch_real", "FETCH_SIZE"), ("write_real", "WRITE_SIZE"), ("fetch_cal", "FETCH_SIZE"),
                      ("write_cal", "WRITE_SIZE")):
        xs = kernel_values(os.path.join(out, name), ctr)
        # last dispatch = a timed launch (warm table, warm caches as in the bench)
        res[name] = xs[-1] * 1024.0 if xs else None
    # L2 hit rate of the same (last, timed) launch: TCC requests that hit
    hits = kernel_values(os.path.join(out, "l2_real"), "TCC_HIT_sum")
    miss = kernel_values(os.path.join(out, "l2_real"), "TCC_MISS_sum")
    l2 = None
    if hits and miss and hits[-1] + miss[-1] > 0:
        l2 = {"hits": hits[-1], "misses": miss[-1], "hit_rate": round(hits[-1] / (hits[-1] + miss[-1]), 4)}
    real = json.load(open(os.path.join(out, "fetch_real.json")))
    cfg = real["config"]
    n_docs, doc_b = cfg["docs_per_gpu"], cfg["doc_bytes"]
    known_read = n_docs * doc_b + 8 * (n_docs + 1)
    known_write = 4 * n_docs
    f_read = known_read / res["fetch_cal"] if res["fetch_cal"] else None
    f_write = known_write / res["write_cal"] if res["write_cal"] else None
    # The empty-table run is the launch's streaming part (documents, offsets),
    # which FETCH_SIZE counts at half (factor f_read, ~2).  What the real run
    # fetches beyond it is table / Bloom gathers: random loads, which
    # FETCH_SIZE counts at one 64-B request each (profiles/r02_gather_cal.json,
    # tools/gather_cal.hip: factor g_read ~1) -- the streaming factor must not
    # be applied to them.
    g_read = 1.0
    cal = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r02_gather_cal.json")
    if os.path.exists(cal):
        fpg = json.load(open(cal)).get("fetch_per_gather_B")
        if fpg:
            g_read = 64.0 / fpg
    traffic = None
    if f_read and f_write:
        stream_part = min(res["fetch_cal"], res["fetch_real"])
        gather_part = res["fetch_real"] - stream_part
        traffic = stream_part * f_read + gather_part * g_read + res["write_real"] * f_write
    wl = real["roofline"].get("workload_key") or (
        f"score:docs={n_docs}:bytes={doc_b}:L={cfg['languages']}:G={','.join(map(str, cfg['gram_lengths']))}"
        f":K={cfg['profile_size']}")
    doc = {"workload_key": wl, "counters_bytes": res, "known_cal_read": known_read, "known_cal_write": known_write,
           "read_factor": f_read, "gather_read_factor": g_read, "write_factor": f_write,
           "traffic_bytes_per_launch": round(traffic) if traffic else None,
           "l2": l2,
           "algorithmic_bytes_per_launch": real["roofline"]["algorithmic_bytes_per_launch"],
           "note": "FETCH_SIZE/WRITE_SIZE (KiB) x 1024; the streaming part calibrated on an empty-table launch of "
                   "the same kernel, the remainder (random gathers) at the gather calibration's factor"}
    with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
