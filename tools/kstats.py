#!/usr/bin/env python3
"""Short per-kernel table of a rocprofv3 kernel_stats.csv: tools/kstats.py FILE [pattern]"""
import csv
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else "ldgpu"
rows = [r for r in csv.DictReader(open(sys.argv[1])) if pat in r["Name"]]
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"])):
    n = r["Name"].split("(ldgpu")[0] if "(ldgpu" in r["Name"] else r["Name"].split("(")[0]
    n = n.replace("ldgpu::(anonymous namespace)::", "").replace("void ", "")
    print(f"{n[:44]:44s} calls={r['Calls']:>5} total_ms={int(r['TotalDurationNs'])/1e6:9.2f} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
