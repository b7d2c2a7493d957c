#!/usr/bin/env python3
"""Plan tuning report: per-rule GPU plan and candidate counts on a synthetic corpus
(emulated kernels on the CPU)."""
import ctypes as C
import sys
import os
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
from trivy_amd import corpus, secret as S, _native as N


def main(mb=64, seed=2, chunk=256):
    b, info = corpus.make_corpus(int(mb) << 20, seed=seed)
    sc = S.NewScanner(None)
    L = N.lib()
    R = len(sc.Rules)
    info_ = sc.info()
    cpr = np.zeros(R, dtype=np.uint64)
    gb = np.zeros(info_["n_groups"], dtype=np.uint64)
    u64p = C.POINTER(C.c_uint64)
    t = time.time()
    N.check(L.tsg_emulate_candidate_stats(sc.handle, C.c_void_p(b.data.ctypes.data),
                                          b.offsets.ctypes.data_as(u64p), b.nfiles, chunk,
                                          cpr.ctypes.data_as(u64p), gb.ctypes.data_as(u64p)))
    print("emulated in %.1fs; corpus %s" % (time.time() - t, info))
    rows = []
    for r in range(R):
        g, rl, ml = C.c_int32(), C.c_int32(), C.c_int64()
        L.tsg_ruleset_rule_plan(sc.handle, r, C.byref(g), C.byref(rl), C.byref(ml))
        rows.append((int(cpr[r]), sc.Rules[r].ID, g.value, rl.value, ml.value,
                     int(gb[g.value]) if g.value >= 0 else -1))
    for row in sorted(rows, reverse=True):
        print("%8d cand  %-32s group=%3d relax=%3d maxlen=%5d gated=%.1f%%" % (
            row[0], row[1], row[2], row[3], row[4], 100.0 * row[5] / info["bytes"]))
    print("total gated bytes over groups: %.2fx corpus" % (gb.sum() / info["bytes"]))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
