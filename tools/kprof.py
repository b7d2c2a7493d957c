#!/usr/bin/env python3
"""One K1+K2 pass over a fixed corpus, for rocprofv3 (kernel trace / PMC passes)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from trivy_amd import corpus, secret as S

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
b, info = corpus.make_corpus(int(gb * (1 << 30)), seed=2)
sc = S.NewScanner(None)
ctx = S.GpuContext(sc, 0)
ctx.upload(b)
for _ in range(reps):
    ctx.kernels()
print(ctx.stats(), flush=True)
ctx.close()
