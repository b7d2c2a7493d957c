#!/usr/bin/env python3
"""Host resolution profile on the GPU box: one scan of a seeded corpus with TSG_PROF=1."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ["TSG_PROF"] = "1"
from trivy_amd import corpus, secret as S, _native as N

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 0
b, info = corpus.make_corpus(int(gb * (1 << 30)), seed=1002, plants_per_mib=1.0)
sc = S.NewScanner(None)
ctx = S.GpuContext(sc, 0, host_threads=nt)
ctx.upload(b)
for i in range(3):
    t = time.perf_counter()
    out = ctx.scan_raw()
    dt = time.perf_counter() - t
    N.lib().tsg_result_free(out)
    st = ctx.stats()
    print("scan %d: wall %.1f ms, resolve %.1f ms, k1 %.2f gate %.2f k2 %.2f" % (
        i, dt * 1e3, st["resolve_ms"], st["k1_ms"], st["gate_ms"], st["k2_ms"]), flush=True)
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
ctx.close()
