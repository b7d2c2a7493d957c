#!/usr/bin/env python3
"""Kernel-only A/B timing on the GPU: one seeded batch, the device part scanned repeatedly
through the synchronous kernels hook; median K1 / gates / K2 HIP-event ms.  Run it once per
library variant (TSG_LIB_VARIANT=<name>, tools/build_variants.sh).

    python tools/kab.py [MiB] [reps] [--rules builtin|user1000|allow-exclude] [--knob name=value]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rules = sys.argv[sys.argv.index("--rules") + 1] if "--rules" in sys.argv else "builtin"
    knobs = [sys.argv[i + 1] for i, a in enumerate(sys.argv) if a == "--knob"]
    args = [a for a in sys.argv[1:] if not a.startswith("--") and a != rules and a not in knobs]
    from trivy_amd import _native as N
    for kv in knobs:  # tsg_test_knob, before the rule set compiles
        N.knob(*kv.split("=", 1))
    mib = int(args[0]) if args else 1024
    reps = int(args[1]) if len(args) > 1 else 7
    from bench import rule_set
    from trivy_amd import corpus
    from trivy_amd import secret as S
    sc, extra, binary_frac, _, _ = rule_set(rules)
    b, info = corpus.make_corpus(mib << 20, seed=2, plants_per_mib=1.0, extra_plants=extra,
                                 extra_per_mib=2.0 if extra else 0.0, binary_frac=binary_frac)
    ctx = S.GpuContext(sc, 0)
    ctx.upload(b)
    ctx.kernels()  # adaptation
    rows = []
    for _ in range(reps):
        ctx.kernels()
        rows.append(ctx.stats())
    ctx.close()
    med = lambda k: statistics.median(r[k] for r in rows)  # noqa: E731
    nb = int(b.offsets[-1])
    out = {"variant": os.environ.get("TSG_LIB_VARIANT", "default"), "bytes": nb, "rules": rules, "knobs": knobs,
           "k1_ms": round(med("k1_ms"), 4), "gate_ms": round(med("gate_ms"), 4),
           "k2_ms": round(med("k2_ms"), 4),
           "k1_clk_ms": round(med("k1_clock_ms"), 4), "chain_clk_ms": round(med("chain_clock_ms"), 4),
           "post_k1_clk_ms": round(med("post_k1_clock_ms"), 4),
           "k1_GBps": round(nb / med("k1_ms") / 1e6, 1),
           "dev_GBps": round(nb / (med("k1_ms") + med("gate_ms") + med("k2_ms")) / 1e6, 1),
           "k2_items": rows[-1]["k2_items"], "k2_entries": rows[-1]["k2_launches"],
           "candidates": rows[-1]["candidates"], "k1x_records": rows[-1]["k1x_records"],
           "k1x_inline": rows[-1]["k1x_inline"],
           "k1f_listed": rows[-1]["k1f_listed"], "event_chunks": rows[-1]["event_chunks"], "k1f_arrivals": rows[-1]["k1f_arrivals"],
           "k1_hot": rows[-1]["k1_hot_states"],
           "diag": [rows[-1]["k2_tail_bytes"], rows[-1]["k2_tail_max"], rows[-1]["k2_long_tails"]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
