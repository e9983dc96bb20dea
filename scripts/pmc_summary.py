"""Summarise rocprofv3 counter CSVs per kernel (per dispatch averages).
usage: python scripts/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_fetch ..."""
import collections
import csv
import os
import sys

for d in sys.argv[1:]:
    path = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    print(f"== {d}")
    for k, v in agg.items():
        n = len(disp[k])
        print(f"  {k} ({n} dispatches): " + ", ".join(f"{a}={b / n:.4g}" for a, b in sorted(v.items())))
