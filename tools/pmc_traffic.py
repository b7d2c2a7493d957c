#!/usr/bin/env python3
"""HBM traffic per launch from a rocprofv3 `--pmc FETCH_SIZE` counter CSV.

    python tools/pmc_traffic.py <counter_collection.csv> [kernel-substring]

FETCH_SIZE is in KiB and, on gfx950, counts half the bytes of a 16-B-per-lane streaming
read (MI355X_MICROARCH.md, HBM section): bytes = FETCH_SIZE * 1024 * 2.  Launches with a
grid below 1/4 of the largest launch of the same kernel (the K1 sampling pass) are skipped.
"""
import csv
import json
import sys


def traffic(path, kernel="k1_kernel"):
    rows = [r for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    if not rows:
        return None
    gmax = max(int(r["Grid_Size"]) for r in rows)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) * 4 >= gmax]
    return sum(vals) / len(vals) * 1024 * 2


if __name__ == "__main__":
    k = sys.argv[2] if len(sys.argv) > 2 else "k1_kernel"
    print(json.dumps({"kernel": k, "bytes_per_launch": traffic(sys.argv[1], k)}))
