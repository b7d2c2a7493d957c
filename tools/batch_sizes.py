#!/usr/bin/env python3
"""Per-batch cost vs batch size on one device: tsg_scan_batch of seeded batches of
1..256 MiB (builtin rules), each timed over several calls after a warm-up; prints one JSON
line per size with ms per batch, GB/s, and the context's K1/K2/resolve times.

    python tools/batch_sizes.py [sizes_mib...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [1, 8, 32, 128, 256]
    import ctypes as C
    from trivy_amd import _native as N
    from trivy_amd import corpus
    from trivy_amd import secret as S
    sc = S.NewScanner(None)
    ctx = S.GpuContext(sc, 0)
    big, _ = corpus.make_corpus(max(sizes) << 20, seed=2, plants_per_mib=1.0)
    # adaptation first (a batch of >= 16 MiB), as in a long-running process
    ctx.scan_batch(big)
    L = N.lib()
    for mib in sizes:
        import numpy as np
        f1 = int(np.searchsorted(big.offsets, mib << 20, side="right")) - 1
        b = S.Batch(big.data[:int(big.offsets[f1])], big.offsets[:f1 + 1], big.paths[:int(big.path_offsets[f1])],
                    big.path_offsets[:f1 + 1])
        reps = max(3, min(40, 512 // mib))
        out = C.c_void_p()
        N.check(L.tsg_scan_batch(ctx.handle, *b.ptrs(), C.byref(out)))
        L.tsg_result_free(out)
        st0 = ctx.stats()
        t0 = time.perf_counter()
        for _ in range(reps):
            N.check(L.tsg_scan_batch(ctx.handle, *b.ptrs(), C.byref(out)))
            L.tsg_result_free(out)
        dt = (time.perf_counter() - t0) / reps
        st = ctx.stats()
        nb = st["batches"] - st0["batches"]
        per = lambda k: round((st[k] - st0[k]) / max(1, nb), 3)  # noqa: E731
        print(json.dumps({"mib": mib, "files": f1, "ms_per_batch": round(dt * 1e3, 3),
                          "GBps": round(int(b.offsets[-1]) / dt / 1e9, 2), "h2d_ms": per("sum_h2d_ms"),
                          "k1_ms": per("sum_k1_ms"), "gate_ms": per("sum_gate_ms"), "k2_ms": per("sum_k2_ms"),
                          "d2h_ms": per("sum_d2h_ms"), "resolve_ms": per("sum_resolve_ms")}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
