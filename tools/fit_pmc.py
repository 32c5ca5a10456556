#!/usr/bin/env python3
"""pmc_traffic_fit*.json from tools/fit_pmc.sh: raw FETCH_SIZE / WRITE_SIZE
(KB) summed per kernel over the run's two counts, calibrated on kernels of
known bytes, per count and per window:
  FIT v4: part2 reads and writes each record once (8 B per corpus byte, K = 1);
  FIT v5: sort_emit writes one 8-B sort key per corpus byte (write factor),
          runs_count reads the sorted keys once (8 B per key; round 5:
          sort_runs, once per gram length).
    python tools/fit_pmc.py OUTDIR [OUTNAME]"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import count_traffic, is_count_kernel  # noqa: E402  (one attribution rule for both)

out = sys.argv[1]
line = json.load(open(os.path.join(out, "WRITE_SIZE.json")))
cfg = line["config"]
counts = 2  # bench --steps 1 --warmup 0: the timed count and the statistics count
raw = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for ln in open(os.path.join(out, ctr + ".sum")):
        k, n, v = ln.rstrip("\n").split("\t")
        raw.setdefault(k, {})[ctr] = float(v) * 1024 / counts
rec_bytes = 8 * cfg["corpus_bytes_per_gpu"]  # K = 1 records / FIT v5 keys: one per byte position
p2 = next((v for k, v in raw.items() if k.startswith("part2_kernel")), None)
if p2:
    rf, wf = rec_bytes / p2["FETCH_SIZE"], rec_bytes / p2["WRITE_SIZE"]
    calibration = "part2 reads and writes every record once (8 B per corpus byte): factors = those bytes / its raw FETCH_SIZE, WRITE_SIZE; applied to every kernel (random probes of merge / derive: approximate)"
else:
    grams = [int(g) for g in re.search(r"grams ([\d,]+),", cfg["workload"]).group(1).split(",")]
    n_len = len({g for g in grams if g <= 7})
    em = next(v for k, v in raw.items() if k.startswith("sort_emit_kernel"))
    rc = next((v for k, v in raw.items() if k.startswith("runs_count_kernel")), None)
    wf = rec_bytes / em["WRITE_SIZE"]
    if rc:  # round 6: one pass counts every length's runs, reading each sorted key once
        rf = 8 * cfg["windows_per_gpu"] / max(1, len(grams)) / rc["FETCH_SIZE"]
        calibration = ("FIT v5: write factor = sort_emit's 8 B per corpus byte / its raw WRITE_SIZE; read factor = "
                       "runs_count's 8 B per sorted key (one pass) / its raw FETCH_SIZE; applied to every kernel "
                       "(the random probes of runs_add into T and the radix sort's scatter: approximate)")
    else:  # round 5: sort_runs read the keys once per gram length
        rn = next(v for k, v in raw.items() if k.startswith("sort_runs_kernel"))
        rf = 8 * cfg["windows_per_gpu"] / max(1, len(grams)) * n_len / rn["FETCH_SIZE"]
        calibration = ("FIT v5: write factor = sort_emit's 8 B per corpus byte / its raw WRITE_SIZE; read factor = "
                       "sort_runs' 8 B per key per gram-length pass / its raw FETCH_SIZE; applied to every kernel "
                       "(the random probes of runs_add into T and the radix sort's scatter: approximate)")
m = re.search(r"(\d+) languages, grams ([\d,]+), profile", cfg["workload"])
L, grams = int(m.group(1)), [int(g) for g in m.group(2).split(",")]
# only the count's own kernels (bench.is_count_kernel): a FIT v4 count sorts
# nothing, so a radix sort of its run belongs to an export or the table phase
own = {k: v for k, v in raw.items() if is_count_kernel(k, L, grams)}
fetch = sum(v.get("FETCH_SIZE", 0.0) for v in own.values())
write = sum(v.get("WRITE_SIZE", 0.0) for v in own.values())
windows = cfg["windows_per_gpu"]
d = {"workload_key": f"fit:bytes={cfg['corpus_bytes_per_gpu']}:L={L}:G={m.group(2)}",
     "per_kernel_raw_bytes_per_count": raw,
     "excluded_kernels": sorted(k for k in raw if k not in own),
     "read_factor": round(rf, 4), "write_factor": round(wf, 4),
     "calibration": calibration, "count_only": True}
traffic = count_traffic(d, L, grams)
d.update({"traffic_bytes_per_launch": traffic, "traffic_raw_bytes_per_count": round(fetch + write),
          "windows_per_count": windows, "bytes_per_window_corrected": round(traffic / windows, 2),
          "bytes_per_window_raw": round((fetch + write) / windows, 2),
          "count_ms": line["roofline"]["count_ms"],
          "memory_side_GBps": round(traffic / (line["roofline"]["count_ms"] * 1e-3) / 1e9, 1)})
json.dump(d, open(os.path.join(out, sys.argv[2] if len(sys.argv) > 2 else "pmc_traffic_fit.json"), "w"), indent=1)
print(json.dumps({k: d[k] for k in d if k != "per_kernel_raw_bytes_per_count"}, indent=1))
for k, v in sorted(raw.items(), key=lambda kv: -sum(kv[1].values())):
    print(f"  {k:32s} fetch {v.get('FETCH_SIZE', 0) / 1e9:8.2f} GB  write {v.get('WRITE_SIZE', 0) / 1e9:8.2f} GB (raw)")
