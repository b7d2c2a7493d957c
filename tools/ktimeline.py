#!/usr/bin/env python3
"""Per-batch kernel timeline from a rocprofv3 kernel trace (csv): for the last batch of the
run (the span from its last prep_kernel to the outputs_kernel after it), each kernel's start
offset, duration and the gap before it, in microseconds.

    python tools/ktimeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows))
    starts = [i for i, k in enumerate(ks) if k[2].endswith("prep_kernel")]
    i0 = starts[-2] if len(starts) > 1 else starts[-1]
    t0, prev = ks[i0][0], ks[i0][0]
    for s, e, n in ks[i0:]:
        print("%9.1f %8.1f %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, n[-60:]))
        prev = e
        if n.endswith("outputs_kernel") and s > ks[i0][0]:
            break


if __name__ == "__main__":
    main()
