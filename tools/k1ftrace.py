#!/usr/bin/env python3
"""K1F per-wave timing (TSG_K1F_TRACE): how the waves of one launch spread out.

    python tools/k1ftrace.py run OUT_DIR [MiB]     (GPU box)
    python tools/k1ftrace.py report OUT_DIR         (anywhere)

`run` scans one seeded configs[1] batch twice through the synchronous kernels hook (the
first also adapts K1F) and keeps the trace of the second: per wave its start (after the
block's staging) and end (wall clock, 100 MHz), its tiles, listed words and hardware ids.
`report` prints the launch span, the wave durations and end times (quantiles), and how the
late waves differ (listed words, XCC).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out, mib=1024):
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "k1ftrace.bin")
    if os.path.exists(path):
        os.remove(path)
    from trivy_amd import corpus
    from trivy_amd import secret as S
    b, _ = corpus.make_corpus(mib << 20, seed=2, plants_per_mib=1.0)
    os.environ["TSG_K1F_TRACE"] = path
    ctx = S.GpuContext(S.NewScanner(None), 0)
    ctx.upload(b)
    ctx.kernels()  # (adaptation)
    os.remove(path)
    ctx.kernels()
    st = ctx.stats()
    ctx.close()
    with open(os.path.join(out, "k1ftrace_stats.json"), "w") as f:
        json.dump({"k1_ms": st["k1_ms"], "bytes": int(b.offsets[-1])}, f)


def report(out):
    t = np.fromfile(os.path.join(out, "k1ftrace.bin"), dtype=np.uint64).reshape(-1, 4)
    slot = (np.arange(len(t)) % 16) // 4  # record = block * 16 + wave; SIMD slot = wave / 4
    keep = t[:, 1] > 0
    t, slot = t[keep], slot[keep]
    s, e = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    t0 = s.min()
    dur, end, start = (e - s) / 100.0, (e - t0) / 100.0, (s - t0) / 100.0  # us
    tiles, listed = (t[:, 2] >> 32).astype(np.int64), (t[:, 2] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 3] >> 32).astype(np.int64) & 0xF
    q = lambda v: [round(float(np.percentile(v, p)), 1) for p in (0, 10, 50, 90, 99, 100)]  # noqa: E731
    rep = {"waves": int(len(t)), "span_us": round(float(end.max()), 1),
           "start_us_q0_10_50_90_99_100": q(start), "dur_us_q": q(dur), "end_us_q": q(end),
           "tiles_q": q(tiles), "listed_q": q(listed)}
    late = end >= np.percentile(end, 95)
    rep["late5pct"] = {"listed_mean": round(float(listed[late].mean()), 1), "listed_mean_all": round(float(listed.mean()), 1),
                       "start_mean_us": round(float(start[late].mean()), 1), "xcc": np.bincount(xcc[late], minlength=8).tolist()}
    rep["end_by_xcc_us"] = [round(float(end[xcc == x].max()), 1) if (xcc == x).any() else None for x in range(8)]
    upt = [float((dur[slot == k] / np.maximum(tiles[slot == k], 1)).mean()) for k in range(4)]
    rep["by_slot"] = {"dur_us": [round(float(dur[slot == k].mean()), 1) for k in range(4)],
                      "end_us_max": [round(float(end[slot == k].max()), 1) for k in range(4)],
                      "us_per_tile": [round(u, 3) for u in upt],
                      "shares_next": [round(1000 * (1 / u) / sum(1 / v for v in upt)) for u in upt]}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1024)
    else:
        report(sys.argv[2])
