#!/usr/bin/env python3
"""HBM traffic per launch from a rocprofv3 `--pmc FETCH_SIZE` counter CSV.

    python tools/pmc_traffic.py <counter_collection.csv> [kernel-substring]
    python tools/pmc_traffic.py --record RULES CSV BENCH_JSON COMMITTED_CSV_PATH > rec.json

--record writes the record bench.py reads from profiles/pmc/<RULES>.json: K1 / K2 HBM bytes
per launch of that pass, the batch size of the bench line of the same run, and the sha256
of the device code that ran (bench.py uses the traffic only while the sources still match).

FETCH_SIZE is in KiB and counts memory-side read requests x 64 B (MI355X_MICROARCH.md, HBM
section), so how many bytes one KiB stands for depends on the request width of the access
pattern: exactly 1/2 for 16-B-per-lane streaming reads (k1f_kernel), 0.92 for the automaton
K1's quad-transposed 64-B segment loads.  The factor per kernel comes from profiles/pmc/fetch_calib.json (a
calibration run on a known byte count, tools/fetch_calib.hip).  Launches with a grid below
1/4 of the largest launch of the same kernel (the K1 sampling pass) are skipped.
"""
import csv
import json
import os
import sys

CALIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc", "fetch_calib.json")


def fetch_factor(kernel):
    """FETCH_SIZE bytes per byte read for the kernel's access pattern."""
    c = json.load(open(CALIB))
    for k, pat in c["kernels"].items():
        if k in kernel:
            return c[pat]
    return c["stream16"]


def traffic(path, kernel="k1_kernel"):
    rows = [r for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    if not rows:
        return None
    gmax = max(int(r["Grid_Size"]) for r in rows)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) * 4 >= gmax]
    return sum(vals) / len(vals) * 1024 / fetch_factor(kernel)


def record(rules, csv_path, bench_json, committed):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import kernel_source_sha
    line = None
    for ln in open(bench_json):
        if ln.startswith("{"):
            line = json.loads(ln)
    k1 = "k1f_kernel" if traffic(csv_path, "k1f_kernel") is not None else "k1_kernel"
    t1 = traffic(csv_path, k1)
    t2 = traffic(csv_path, "k2_kernel")
    return {"rules": rules, "batch_bytes": line["roofline"]["algorithmic_bytes_per_launch"],
            "kernels_sha256": kernel_source_sha(), "csv": committed, "k1_kernel": k1,
            "fetch_factor": fetch_factor(k1),
            "k1_bytes_per_launch": None if t1 is None else int(t1),
            "k2_bytes_per_launch": None if t2 is None else int(t2),
            "k2_item_bytes_last_batch": line["kernels"]["k2_item_bytes_last_batch"]}


if __name__ == "__main__":
    if sys.argv[1] == "--record":
        print(json.dumps(record(*sys.argv[2:6]), indent=1))
        sys.exit(0)
    k = sys.argv[2] if len(sys.argv) > 2 else "k1_kernel"
    print(json.dumps({"kernel": k, "bytes_per_launch": traffic(sys.argv[1], k)}))
