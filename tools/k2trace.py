#!/usr/bin/env python3
"""K2 per-entry timing (TSG_K2_TRACE): where the list kernel's time goes.

    python tools/k2trace.py run OUT_DIR [MiB] [--rules builtin|user1000]   (GPU box)
    python tools/k2trace.py report OUT_DIR                                  (anywhere)

`run` scans one seeded batch twice through the synchronous kernels hook (the first scan
also adapts K1) and keeps the trace of the second: per list entry the wall-clock start and
end (100 MHz), its group and item count, and the XCC / hardware id of the block that ran
it.  `report` summarises it: kernel span, entry durations, the tail after most blocks have
finished, the slowest entries and groups, and per-XCC busy time.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out, mib=1024, rules="builtin"):
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "k2trace.bin")
    if os.path.exists(path):
        os.remove(path)
    from bench import rule_set
    from trivy_amd import corpus
    from trivy_amd import secret as S
    sc, extra, binary_frac, _, _ = rule_set(rules)
    b, info = corpus.make_corpus(mib << 20, seed=2, plants_per_mib=1.0, extra_plants=extra,
                                 extra_per_mib=2.0 if extra else 0.0, binary_frac=binary_frac)
    os.environ["TSG_K2_TRACE"] = path  # (read once, at the first batch)
    ctx = S.GpuContext(sc, 0)
    ctx.upload(b)
    ctx.kernels()  # (adaptation)
    os.remove(path)
    ctx.kernels()
    st = ctx.stats()
    ctx.close()
    meta = {"bytes": int(b.offsets[-1]), "files": b.nfiles, "rules": rules,
            "k2_ms": st["k2_ms"], "k1_ms": st["k1_ms"], "gate_ms": st["gate_ms"],
            "k2_items": st["k2_items"], "k2_entries": st["k2_launches"]}
    json.dump(meta, open(os.path.join(out, "k2trace_meta.json"), "w"), indent=1)
    print(json.dumps(meta))


def report(out):
    meta = json.load(open(os.path.join(out, "k2trace_meta.json")))
    t = np.fromfile(os.path.join(out, "k2trace.bin"), dtype=np.uint64).reshape(-1, 8)
    t = t[t[:, 0] > 0]
    st, en = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    en = np.where(en > 0, en, st)
    g = (t[:, 2] >> 32).astype(np.int64)
    n = (t[:, 2] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 3] >> 32).astype(np.int64) & 0xF
    t0 = st.min()
    us = lambda x: x * 0.01  # 100 MHz ticks -> us  # noqa: E731
    dur = us(en - st)
    span = us(en.max() - t0)
    order = np.argsort(-dur)
    rep = {"meta": meta, "entries": int(len(t)), "span_us": round(float(span), 1),
           "dur_us": {k: round(float(np.percentile(dur, p)), 2) for k, p in
                      (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
           "sum_dur_us": round(float(dur.sum()), 1),
           "start_us": {k: round(float(np.percentile(us(st - t0), p)), 2) for k, p in
                        (("p50", 50), ("p90", 90), ("max", 100))},
           "end_us": {k: round(float(np.percentile(us(en - t0), p)), 2) for k, p in
                      (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
           "slowest": [{"group": int(g[i]), "items": int(n[i]), "dur_us": round(float(dur[i]), 1),
                        "start_us": round(float(us(st[i] - t0)), 1), "xcc": int(xcc[i]),
                        "replays": int(t[i, 4]), "cands": int(t[i, 5]), "tail_bytes": int(t[i, 6]),
                        "tail_max": int(t[i, 7])}
                       for i in order[:15]],
           # per-entry counters (K2_TRACE_CTR builds; zero otherwise)
           "counters_total": {"replays": int(t[:, 4].sum()), "cands": int(t[:, 5].sum()),
                              "tail_bytes": int(t[:, 6].sum()), "tail_max": int(t[:, 7].max())}}
    per_g = {}
    for i in range(len(t)):
        d = per_g.setdefault(int(g[i]), [0, 0.0, 0.0])
        d[0] += int(n[i])
        d[1] += float(dur[i])
        d[2] = max(d[2], float(dur[i]))
    rep["groups_by_time"] = sorted(({"group": k, "items": v[0], "sum_us": round(v[1], 1),
                                     "max_us": round(v[2], 1)} for k, v in per_g.items()),
                                   key=lambda x: -x["sum_us"])[:15]
    rep["us_per_item"] = {k: round(float(np.percentile(dur / np.maximum(n, 1), p)), 3)
                          for k, p in (("p50", 50), ("p90", 90), ("max", 100))}
    rep["busy_us_per_xcc"] = {int(x): round(float(dur[xcc == x].sum()), 1) for x in np.unique(xcc)}
    if "--phases" in sys.argv:  # K2_TRACE_PHASE builds: thread 0's stamps in words 4..7
        ph = t[:, 4:8].astype(np.int64)
        ok = (ph > 0).all(axis=1)
        marks = np.column_stack([st, ph, en])[ok]
        names = ["claim..staged", "staged..setup", "setup..loop", "loop..tails", "tails..next claim"]
        rep["phases_us_p50"] = {nm: round(float(np.median(us(marks[:, i + 1] - marks[:, i]))), 2)
                                for i, nm in enumerate(names)}
        rep["phases_us_mean"] = {nm: round(float(np.mean(us(marks[:, i + 1] - marks[:, i]))), 2)
                                 for i, nm in enumerate(names)}
    print(json.dumps(rep, indent=1))
    return rep


if __name__ == "__main__":
    if sys.argv[1] == "run":
        rules = sys.argv[sys.argv.index("--rules") + 1] if "--rules" in sys.argv else "builtin"
        args = [a for a in sys.argv[3:] if not a.startswith("--") and a != rules]
        run(sys.argv[2], int(args[0]) if args else 1024, rules)
    else:
        report(sys.argv[2])
