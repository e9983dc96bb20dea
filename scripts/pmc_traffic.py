"""Per-dispatch HBM traffic of each kernel from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md HBM section).
FETCH_SIZE and WRITE_SIZE are in KiB; reported here in bytes.  FETCH_SIZE is
corrected x2: tools/fetch_calib.hip measured FETCH_SIZE = RDREQ x 64 B with
every request a 128-B line for each access pattern the kernels use (16-B and
8-B coalesced, record pairs, unaligned windows, random 16-B gathers;
profiles/r3_fetch_calibration.txt).  WRITE_SIZE is exact for 16-B stores.
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
       "correction": "fetch = 2 x FETCH_SIZE (profiles/r3_fetch_calibration.txt); write = WRITE_SIZE",
       "kernels": {k: {"fetch_size_raw": fetch.get(k), "fetch": 2 * (fetch.get(k) or 0), "write": write.get(k),
                       "traffic": 2 * (fetch.get(k) or 0) + (write.get(k) or 0)}
                   for k in sorted(set(fetch) | set(write)) if k.startswith("zd_k_")}}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
