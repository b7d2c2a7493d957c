#!/usr/bin/env python3
"""Plan tuning report: per-rule GPU plan (anchor event, group, relaxation) and candidate
counts, plus the bytes K2 scans per group, on a synthetic corpus (emulated kernels, CPU).

    python tools/plan_stats.py [MiB] [seed] [chunk]
"""
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
    print("emulated in %.1fs; corpus %s; plan %s" % (time.time() - t, info, info_))
    rows = []
    for r in range(R):
        g, rl, ml = C.c_int32(), C.c_int32(), C.c_int64()
        L.tsg_ruleset_rule_plan(sc.handle, r, C.byref(g), C.byref(rl), C.byref(ml))
        ev, ed = C.c_uint32(), C.c_int64()
        desc = C.create_string_buffer(128)
        L.tsg_ruleset_rule_anchor(sc.handle, r, C.byref(ev), C.byref(ed), desc, 128)
        rows.append((int(cpr[r]), sc.Rules[r].ID, g.value, rl.value, ml.value,
                     int(gb[g.value]) if g.value >= 0 else -1, ev.value, ed.value, desc.value.decode()))
    for row in sorted(rows, reverse=True):
        print("%7d cand %-30s g=%3d relax=%3d maxlen=%5d k2=%6.2f%% ev=%08x d=%4d %s" % (
            row[0], row[1], row[2], row[3], row[4], 100.0 * row[5] / info["bytes"], row[6], row[7], row[8]))
    print("K2 bytes over all groups: %.4fx corpus" % (gb.sum() / info["bytes"]))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
