"""profiles/pmc_traffic_fit.json from a tools/pmc_profile.sh FETCH_SIZE /
WRITE_SIZE run of the fit bench (one count = the dispatches of one batch
loop): per-kernel raw KB per dispatch, corrected HBM bytes per count.

    python tools/fit_traffic.py gpurun_out/pmcfitN/summary.txt DISPATCHES_PER_COUNT
"""
import json
import re
import sys

WINDOWS = 5366581155  # bench.py --mode fit default corpus (1 GiB, grams 1-5)


def main(summary, per_count):
    raw, k = {}, None
    for line in open(summary):
        m = re.match(r"ldgpu::\(anonymous namespace\)::(\w+)\(", line)
        if m:
            k = m.group(1)
            continue
        m = re.match(r"\s+(FETCH_SIZE|WRITE_SIZE)\s+mean/dispatch\s+([\d.]+)", line)
        if m and k:
            raw.setdefault(k, {})[m.group(1)] = float(m.group(2))
    fetch = sum(v.get("FETCH_SIZE", 0.0) for v in raw.values()) * 1024 * per_count
    write = sum(v.get("WRITE_SIZE", 0.0) for v in raw.values()) * 1024 * per_count
    d = {"workload_key": "fit:bytes=1073841929:L=20:G=1,2,3,4,5",
         "per_kernel_raw_kb_per_dispatch": raw, "dispatches_per_count": per_count,
         "fetch_raw_bytes_per_count": fetch, "write_raw_bytes_per_count": write,
         "read_factor": 2.0,
         "read_factor_note": "FETCH_SIZE reports 1/2 of streaming-read bytes on gfx950 (MI355X_MICROARCH.md); "
                             "checked on reduce_kernel, which reads its records exactly once. Applied to every FIT "
                             "kernel's fetch (merge's random probes included: an upper bound)",
         "traffic_bytes_per_launch": 2 * fetch + write, "traffic_raw_bytes_per_count": fetch + write,
         "windows_per_count": WINDOWS,
         "bytes_per_window_corrected": round((2 * fetch + write) / WINDOWS, 2),
         "bytes_per_window_raw": round((fetch + write) / WINDOWS, 2),
         "round1_bytes_per_window": 55.7,
         "command": "ONLY=\"4 5\" tools/pmc_profile.sh gpurun_out/pmcfit --mode fit --steps 1 --warmup 0 --no-cpu-baseline"}
    json.dump(d, open("profiles/pmc_traffic_fit.json", "w"), indent=1)
    print(d["bytes_per_window_corrected"], d["bytes_per_window_raw"], round(d["traffic_bytes_per_launch"] / 1e9, 2))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
