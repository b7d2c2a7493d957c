#!/usr/bin/env python3
"""Kernel-only timing sweep on the GPU (K1 / K2 HIP-event times per chunk size)."""
import json
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from trivy_amd import corpus, secret as S


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    chunks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [256]
    b, info = corpus.make_corpus(int(gb * (1 << 30)), seed=2)
    sc = S.NewScanner(None)
    for ch in chunks:
        ctx = S.GpuContext(sc, 0, chunk_bytes=ch)
        ctx.upload(b)
        ctx.kernels()
        best = None
        for _ in range(3):
            ctx.kernels()
            st = ctx.stats()
            if best is None or st["k1_ms"] + st["k2_ms"] < best["k1_ms"] + best["k2_ms"]:
                best = st
        t = time.perf_counter()
        ctx.scan_raw()
        e2e = time.perf_counter() - t
        st = ctx.stats()
        print(json.dumps({"chunk": ch, "k1_ms": round(best["k1_ms"], 3), "k2_ms": round(best["k2_ms"], 3),
                          "gate_ms": round(best["gate_ms"], 3), "items": best["k2_items"],
                          "k2_bytes": best["k2_bytes"],
                          "k1_GBps": round(info["bytes"] / best["k1_ms"] / 1e6, 1),
                          "resolve_ms": round(st["resolve_ms"], 1), "e2e_ms": round(e2e * 1e3, 1),
                          "cands": st["candidates"], "launches": st["k2_launches"]}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
