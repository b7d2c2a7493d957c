#!/usr/bin/env python3
"""Sanitizer builds of the host C++ (CPU only; never run on the GPU box).

    python tools/sanitize.py thread|address [--run]

Compiles every library source with the sanitizer on the host side only (hipcc
`-Xarch_host -fsanitize=...`; device code is untouched) into trivy_amd/build/san-<kind>/,
links tests/native/stress.cpp against the objects, and with --run executes it on a seeded
corpus with the builtin rules (emulated contexts: slots, lanes, tickets, queue and the
multi-context dispatcher, from 16 threads).  tests/test_sanitizers.py drives this.
"""
import glob
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trivy_amd import build as B  # noqa: E402

FLAGS = {"thread": ["-Xarch_host", "-fsanitize=thread"],
         "address": ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]}
LINK = {"thread": ["-fsanitize=thread", "-fno-gpu-sanitize"],
        "address": ["-fsanitize=address", "-fno-gpu-sanitize"]}


def build(kind):
    out = os.path.join(B.OBJ, "san-" + kind)
    os.makedirs(out, exist_ok=True)
    cxx = ["-O1", "-g", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include")]
    newest_hdr = B._newest(B._headers())

    def comp(src):
        obj = os.path.join(out, os.path.basename(src) + ".o")
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_hdr):
            return obj
        lang = ["--offload-arch=" + B.ARCH, "-x", "hip"] if src.endswith(".hip") else []
        cmd = [B.HIPCC] + lang + cxx + FLAGS[kind] + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stderr))
        return obj

    srcs = B._sources() + [os.path.join(ROOT, "tests", "native", "stress.cpp")]
    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, srcs))
    exe = os.path.join(out, "stress")
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(o) for o in objs):
        cmd = [B.HIPCC, "--offload-arch=" + B.ARCH] + LINK[kind] + ["-o", exe] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stderr))
    return exe


def write_inputs(d, nbytes=3 << 20, seed=9):
    """The builtin rules in the stress driver's line format and a seeded corpus."""
    import numpy as np
    from trivy_amd import corpus
    from trivy_amd import secret as S
    os.makedirs(d, exist_ok=True)
    rules, allow = S.builtin_rules()
    na = lambda v: "-" if v is None else v  # noqa: E731
    with open(os.path.join(d, "rules.txt"), "w") as f:
        for r in rules:
            f.write("\x1f".join([r.ID, r.Category, r.Title, r.Severity, r.Regex,
                                 "\x1e".join(r.Keywords), r.SecretGroupName]) + "\n")
        for a in allow:
            f.write("\x1f".join(["ALLOW", a.ID, a.Description, na(a.Regex), na(a.Path)]) + "\n")
    from trivy_amd import configs
    with open(os.path.join(d, "layer.tar"), "wb") as f:  # pipelined layer / tree scans
        f.write(configs.layer_tar(nbytes // 2, seed=seed, binary_frac=0.05))
    if not os.path.isdir(os.path.join(d, "tree")):
        configs.source_tree(os.path.join(d, "tree"), nbytes // 2, seed=seed)
    b = corpus.fold_runes_batch(seed, nbytes=nbytes, plants=200, frac=0.05)
    b.data.tofile(os.path.join(d, "data.bin"))
    np.asarray(b.offsets, dtype=np.uint64).tofile(os.path.join(d, "offsets.bin"))
    b.paths.tofile(os.path.join(d, "paths.bin"))
    np.asarray(b.path_offsets, dtype=np.uint64).tofile(os.path.join(d, "path_offsets.bin"))
    return os.path.join(d, "rules.txt"), d


def run(kind, workdir, nbytes=3 << 20):
    exe = build(kind)
    rules, d = write_inputs(workdir, nbytes)
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1 halt_on_error=1"
    r = subprocess.run([exe, rules, d], capture_output=True, text=True, env=env, timeout=900)
    return r.returncode, r.stdout + r.stderr


if __name__ == "__main__":
    kind = sys.argv[1]
    if "--run" in sys.argv:
        rc, log = run(kind, "/tmp/tsg_stress_" + kind)
        print(log)
        print(json.dumps({"sanitizer": kind, "rc": rc}))
        sys.exit(rc)
    print(build(kind))
