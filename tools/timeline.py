#!/usr/bin/env python3
"""Device timeline of a bench run from rocprofv3 --kernel-trace --memory-copy-trace CSVs:
per-engine busy time (union of intervals) over the window of the last N big H2D copies,
and how much of the kernels' time overlaps an H2D.

    python tools/timeline.py <dir with run_kernel_trace.csv, run_memory_copy_trace.csv> [min_copy_MB]
"""
import csv
import os
import sys


def union(iv):
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    return tot + (cur[1] - cur[0] if cur else 0)


def overlap(a, b):
    """time of union(a) that also lies in union(b)"""
    ev = sorted([(x, 1, 0) for x, _ in a] + [(y, -1, 0) for _, y in a] +
                [(x, 1, 1) for x, _ in b] + [(y, -1, 1) for _, y in b])
    cnt = [0, 0]
    t0, tot = None, 0
    for t, d, k in ev:
        if t0 is not None and cnt[0] > 0 and cnt[1] > 0:
            tot += t - t0
        cnt[k] += d
        t0 = t
    return tot


def main(d, min_mb=64.0):
    ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    ms = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))))
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ks]
    h2d = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ms
           if r["Direction"].endswith("HOST_TO_DEVICE")]
    # big copies = batch uploads; their size is not in the CSV, so use duration vs the median
    durs = sorted(b - a for a, b in h2d)
    big = [x for x in h2d if x[1] - x[0] >= max(1, durs[len(durs) // 2]) * 50] if durs else []
    big.sort()
    if not big:
        print("no batch uploads found")
        return
    # window: the last step = the last `n` uploads, n = uploads per step (half of all when
    # warmup == steps == 1)
    n = len(big) // 2 if len(big) >= 2 else len(big)
    w = big[-n:]
    lo, hi = w[0][0], max(max(b for _, b in w), max(b for a, b, _ in kern if a >= w[0][0]))
    kin = [(a, b) for a, b, _ in kern if a >= lo and b <= hi]
    k1 = [(a, b) for a, b, nm in kern if a >= lo and b <= hi and "k1_kernel" in nm]
    span = hi - lo
    print("window %.2f ms, %d batch uploads" % (span / 1e6, len(w)))
    print("H2D busy %.2f ms (%.0f%%), kernels busy %.2f ms (%.0f%%), K1 %.2f ms" % (
        union(w) / 1e6, 100 * union(w) / span, union(kin) / 1e6, 100 * union(kin) / span,
        union(k1) / 1e6))
    print("kernel time overlapping an H2D: %.2f ms of %.2f ms" % (overlap(kin, w) / 1e6, union(kin) / 1e6))
    for a, b in w:
        print("  upload %.3f-%.3f ms (%.2f ms)" % ((a - lo) / 1e6, (b - lo) / 1e6, (b - a) / 1e6))


if __name__ == "__main__":
    main(sys.argv[1], *[float(x) for x in sys.argv[2:]])
