#!/usr/bin/env python3
"""Average PMC counters per launch for each kernel from rocprofv3 csv passes
(gpurun_out/prof/pmc_*/run_counter_collection.csv) -> JSON on stdout."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for (k, c), v in sorted(agg.items()):
    out.setdefault(k, {})[c] = sum(v) / len(v)
json.dump(out, sys.stdout, indent=1)
