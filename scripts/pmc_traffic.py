"""Per-dispatch HBM traffic of each kernel from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md HBM section).
FETCH_SIZE and WRITE_SIZE are in KiB; reported here in bytes, uncorrected
(the guide's x2 for FETCH_SIZE holds for 16-B/lane coalesced streaming reads
only; these kernels mix 8-B and unaligned 16-B accesses).
usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [commit]"""
import collections
import csv
import json
import os
import sys


def per_dispatch(d, counter):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("zd::", "")
        agg[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = collections.defaultdict(float)
    for k in agg:                                  # zd_k_tables<false> + <true>: one pass each
        out[k.split("<")[0]] += agg[k] / len(disp[k]) * 1024.0
    return dict(out)


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
out = {"commit": sys.argv[4] if len(sys.argv) > 4 else None, "unit": "bytes per dispatch",
       "kernels": {k: {"fetch": fetch.get(k), "write": write.get(k),
                       "traffic": (fetch.get(k) or 0) + (write.get(k) or 0)}
                   for k in sorted(set(fetch) | set(write)) if k.startswith("zd_k_")}}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
