#!/usr/bin/env python3
"""profiles/pmc_traffic_fit.json from tools/fit_pmc.sh: raw FETCH_SIZE /
WRITE_SIZE (KB) summed per kernel over the run's two counts, calibrated on
part2 (reads and writes each record once: K u64 words per corpus byte), per
count and per window.   python tools/fit_pmc.py OUTDIR"""
import json
import os
import re
import sys

out = sys.argv[1]
line = json.load(open(os.path.join(out, "WRITE_SIZE.json")))
cfg = line["config"]
counts = 2  # bench --steps 1 --warmup 0: the timed count and the statistics count
raw = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for ln in open(os.path.join(out, ctr + ".sum")):
        k, n, v = ln.rstrip("\n").split("\t")
        raw.setdefault(k, {})[ctr] = float(v) * 1024 / counts
rec_bytes = 8 * cfg["corpus_bytes_per_gpu"]  # K = 1 records, one per byte position
p2 = next(v for k, v in raw.items() if k.startswith("part2_kernel"))
rf, wf = rec_bytes / p2["FETCH_SIZE"], rec_bytes / p2["WRITE_SIZE"]
fetch = sum(v.get("FETCH_SIZE", 0.0) for v in raw.values())
write = sum(v.get("WRITE_SIZE", 0.0) for v in raw.values())
traffic = fetch * rf + write * wf
windows = cfg["windows_per_gpu"]
m = re.search(r"(\d+) languages, grams ([\d,]+), profile", cfg["workload"])
d = {"workload_key": f"fit:bytes={cfg['corpus_bytes_per_gpu']}:L={m.group(1)}:G={m.group(2)}",
     "per_kernel_raw_bytes_per_count": raw,
     "read_factor": round(rf, 4), "write_factor": round(wf, 4),
     "calibration": "part2 reads and writes every record once (8 B per corpus byte): factors = those bytes / its raw FETCH_SIZE, WRITE_SIZE; applied to every kernel (random probes of merge / derive: approximate)",
     "traffic_bytes_per_launch": round(traffic), "traffic_raw_bytes_per_count": round(fetch + write),
     "windows_per_count": windows, "bytes_per_window_corrected": round(traffic / windows, 2),
     "bytes_per_window_raw": round((fetch + write) / windows, 2),
     "count_ms": line["roofline"]["count_ms"],
     "memory_side_GBps": round(traffic / (line["roofline"]["count_ms"] * 1e-3) / 1e9, 1)}
json.dump(d, open(os.path.join(out, "pmc_traffic_fit.json"), "w"), indent=1)
print(json.dumps({k: d[k] for k in d if k != "per_kernel_raw_bytes_per_count"}, indent=1))
for k, v in sorted(raw.items(), key=lambda kv: -sum(kv[1].values())):
    print(f"  {k:32s} fetch {v.get('FETCH_SIZE', 0) / 1e9:8.2f} GB  write {v.get('WRITE_SIZE', 0) / 1e9:8.2f} GB (raw)")
