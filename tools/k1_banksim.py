#!/usr/bin/env python3
"""K1 LDS bank-conflict simulation on the CPU (tools/k1_banksim.cpp).

    python tools/k1_banksim.py [MiB] [waves] [--rules builtin|user1000|allow-exclude]

Prints extra LDS cycles per wave instruction for K1's class read and transition read
(current layout and candidate layouts), the share of lanes in the start state, and the
distinct states / dwords per 32-lane half.  Compare with SQ_LDS_BANK_CONFLICT /
SQ_INSTS_LDS of the same kernel (profiles/r03/d1).
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rules = sys.argv[sys.argv.index("--rules") + 1] if "--rules" in sys.argv else "builtin"
    args = [a for a in sys.argv[1:] if not a.startswith("--") and a != rules]
    mib = int(args[0]) if args else 64
    waves = int(args[1]) if len(args) > 1 else 64
    from bench import rule_set
    from trivy_amd import _native as N
    from trivy_amd import corpus
    lib = N.lib()  # noqa: F841  (the tool resolves its symbols against the loaded library)
    so = "/tmp/k1_banksim.so"
    src = os.path.join(ROOT, "tools", "k1_banksim.cpp")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + ROOT + "/include",
                               "-D__HIP_PLATFORM_AMD__", src, "-o", so,
                               os.path.join(ROOT, "trivy_amd", "libtrivy_secret.so")])
    sim = C.CDLL(so)
    sc, extra, bf, _, _ = rule_set(rules)
    b, _ = corpus.make_corpus(mib << 20, seed=2, plants_per_mib=1.0, extra_plants=extra,
                              extra_per_mib=2.0 if extra else 0.0, binary_frac=bf)
    out = (C.c_double * 16)()
    sim.k1_banksim(sc.handle, C.c_void_p(b.data.ctypes.data), C.c_uint64(int(b.offsets[-1])),
                   C.c_uint32(waves), out, 16)
    keys = ["half_steps", "cls_extra_per_inst", "cls_u8x4_extra_per_inst", "tab_extra_per_inst",
            "tab_extra_start_shortcut", "tab_extra_hot8_shortcut", "lanes_in_start",
            "distinct_states_per_half", "distinct_tab_dwords_per_half", "states", "classes"]
    print(json.dumps({k: round(out[i], 3) for i, k in enumerate(keys)}))


if __name__ == "__main__":
    main()
