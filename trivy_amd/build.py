"""Build libtrivy_secret.so in-tree (hipcc, gfx950).

    python -m trivy_amd.build            # incremental
    python -m trivy_amd.build --force

Host C++ (regex engine, DFA compiler, exact resolver) and the HIP kernels are linked
into one shared library whose C ABI is include/trivy_secret.h.  Objects are cached
under trivy_amd/build/ and rebuilt when a source or header is newer.
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libtrivy_secret.so")
ARCH = os.environ.get("TSG_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-I" + os.path.join(ROOT, "include")]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "*.hip")))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(CSRC, "*.inc"))
                  + glob.glob(os.path.join(ROOT, "include", "*.h")))


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0)


def _compile(src, force):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(
            os.path.getmtime(src), _newest(_headers())):
        return obj
    if src.endswith(".hip"):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-x", "hip"] + CXXFLAGS + ["-c", src, "-o", obj]
    else:
        cmd = [HIPCC] + CXXFLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return obj


def build(force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < _newest(objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
