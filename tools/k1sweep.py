#!/usr/bin/env python3
"""K1 block-shape sweep on the GPU: K1 HIP-event time per TSG_K1_CFG (one corpus)."""
import json
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from trivy_amd import corpus, secret as S

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3"]
b, info = corpus.make_corpus(int(gb * (1 << 30)), seed=2)
if os.environ.get("K1SWEEP_BIG"):  # same bytes, re-cut into files of K1SWEEP_BIG bytes
    import numpy as np
    fsz = int(os.environ["K1SWEEP_BIG"])
    n = info["bytes"] // fsz
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(fsz)
    paths = np.frombuffer(b"".join(b"big/%d.txt" % i for i in range(n)), dtype=np.uint8)
    plen = np.array([len(b"big/%d.txt" % i) for i in range(n)], dtype=np.uint64)
    poffs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(plen, out=poffs[1:])
    b = S.Batch(b.data[:n * fsz], offs, paths, poffs)
    info = {"bytes": n * fsz}
sc = S.NewScanner(None)
for cfg in cfgs:
    os.environ["TSG_K1_CFG"] = cfg
    ctx = S.GpuContext(sc, 0)
    ctx.upload(b)
    ctx.kernels()
    best = None
    for _ in range(4):
        ctx.kernels()
        st = ctx.stats()
        best = st["k1_ms"] if best is None else min(best, st["k1_ms"])
    print(json.dumps({"variant": os.environ.get("TSG_LIB_VARIANT", "u8"), "cfg": cfg,
                      "k1_ms": round(best, 3), "k1_GBps": round(info["bytes"] / best / 1e6, 1)}), flush=True)
    ctx.close()
