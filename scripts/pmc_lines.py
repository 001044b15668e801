#!/usr/bin/env python3
"""Per-launch PMC counters of the main match kernel from one rocprofv3 pass
directory, and per topic (launches over the whole batch only).
usage: pmc_lines.py <pass dir> [topics=100000000] [kernel=k_match_fused]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
topics = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
kern = sys.argv[3] if len(sys.argv) > 3 else "k_match_fused"
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and int(r["Grid_Size"]) >= topics // 2:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("  " + ", ".join(f"{c} {sum(v) / len(v) / topics:.3f}/topic" for c, v in sorted(agg.items())))
