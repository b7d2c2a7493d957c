#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc counter CSV (run_counter_collection.csv), over the
full-size dispatches of each kernel (grids below 1/4 of the kernel's largest are sampling
passes and are skipped), plus the derived K1 ratios used in DESIGN.md.

    python tools/sq_summary.py COUNTER_CSV [kernel-substring] [--bytes N]
"""
import collections
import csv
import json
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    nbytes = int(sys.argv[sys.argv.index("--bytes") + 1]) if "--bytes" in sys.argv else 0
    if nbytes:
        args = [a for a in args if a != str(nbytes)]
    path, sub = args[0], (args[1] if len(args) > 1 else "")
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    big = collections.defaultdict(int)
    for r in rows:
        big[r["Kernel_Name"]] = max(big[r["Kernel_Name"]], int(r["Grid_Size"]))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        if int(r["Grid_Size"]) * 4 < big[r["Kernel_Name"]]:
            continue
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        if nbytes and "SQ_INSTS_LDS" in m:
            # SQ_INSTS_* count wave instructions; x64 lanes / bytes
            m["lds_instr_per_byte_lane"] = m["SQ_INSTS_LDS"] * 64 / nbytes
        if nbytes and "SQ_INSTS_VALU" in m:
            m["valu_lane_ops_per_byte"] = m["SQ_INSTS_VALU"] * 64 / nbytes
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_INSTS_LDS" in m and m["SQ_INSTS_LDS"]:
            m["conflict_cycles_per_lds_instr"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            m["wait_any_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        out[k[:80]] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
