"""Mirror of trivy's secret analyzer (pkg/fanal/analyzer/secret/secret.go) and the
binary gate (pkg/fanal/utils/utils.go:71-89), with a batched Analyze for the GPU.

  SecretAnalyzer.Init(configPath)          secret.go:62-76
  SecretAnalyzer.Required(path, size)      secret.go:112-150
  SecretAnalyzer.Analyze(input)            secret.go:78-110   (one file, exact CPU path)
  SecretAnalyzer.AnalyzeBatch(inputs, ...) the batching boundary of SURVEY.md §8f-1:
                                           the same per-file semantics, files scanned
                                           together by the MI355X kernels
  sort_secrets(secrets)                    AnalysisResult.Sort, analyzer.go:212-223
"""
from dataclasses import dataclass

from . import secret as S

VERSION = 1  # secret.go:24 (part of the cache key)

SKIP_FILES = ["go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml",
              "Pipfile.lock", "Gemfile.lock"]
SKIP_DIRS = [".git", "node_modules"]
SKIP_EXTS = [".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb", ".rpm",
             ".zip", ".gz", ".gzip", ".tar", ".pyc"]


def IsBinary(content, file_size):
    """utils.go:71-89: a control byte in the first min(size, 300) bytes."""
    for b in content[:min(file_size, 300)]:
        if b < 7 or b == 11 or (13 < b < 27) or (27 < b < 0x20) or b == 0x7F:
            return True
    return False


def _base(p):
    if p == "":
        return "."
    p = p.rstrip("/")
    if p == "":
        return "/"
    return p[p.rfind("/") + 1:]


def _ext(name):
    i = name.rfind(".")
    return name[i:] if i > name.rfind("/") else ""


@dataclass
class AnalysisInput:
    Dir: str
    FilePath: str
    Content: bytes


class SecretAnalyzer:
    def __init__(self, scanner=None, config_path=""):
        self.scanner = scanner
        self.configPath = config_path

    def Init(self, config_path):
        self.scanner = S.NewScanner(S.ParseConfig(config_path))
        self.configPath = config_path

    def Type(self):
        return "secret"

    def Version(self):
        return VERSION

    def Required(self, file_path, size):
        if size < 10:
            return False
        k = file_path.rfind("/")
        d, name = file_path[:k + 1], file_path[k + 1:]
        dirs = d.split("/")
        if any(sd in dirs for sd in SKIP_DIRS):
            return False
        if name in SKIP_FILES:
            return False
        if _base(self.configPath) == file_path:
            return False
        if _ext(name) in SKIP_EXTS:
            return False
        if self.scanner.AllowPath(file_path):
            return False
        return True

    @staticmethod
    def _scan_path(inp):
        # Files extracted from an image have an empty Dir and no "/" prefix (secret.go:90-96)
        return "/" + inp.FilePath if inp.Dir == "" else inp.FilePath

    def Analyze(self, inp):
        if IsBinary(inp.Content, len(inp.Content)):
            return None
        res = self.scanner.Scan(S.ScanArgs(self._scan_path(inp), inp.Content))
        if not res["Findings"]:
            return None
        return {"Secrets": [res]}

    def AnalyzeBatch(self, inputs, device=None, ctx=None):
        """Analyze many files at once; returns the merged, sorted AnalysisResult.Secrets."""
        args = [S.ScanArgs(self._scan_path(i), i.Content) for i in inputs
                if not IsBinary(i.Content, len(i.Content))]
        res = self.scanner.ScanBatch(args, device=device, ctx=ctx)
        secrets = [r for r in res if r["Findings"]]
        return sort_secrets(secrets)


def _go_sort(items, key, secondary=None):
    """sort.Slice (Go 1.19 pdqsort_func, unstable) of `items` in place by (key bytes,
    secondary): the native restatement in libtrivy_secret.so (tsg_go_sort_perm)."""
    import ctypes as C
    import numpy as np
    from . import _native as N
    n = len(items)
    if n < 2:
        return
    ks = [key(x) for x in items]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(k) for k in ks], out=offs[1:])
    blob = np.frombuffer(b"".join(ks) or b"\0", dtype=np.uint8)
    sec = None if secondary is None else np.array([secondary(x) for x in items], dtype=np.int64)
    perm = np.zeros(n, dtype=np.uint32)
    N.check(N.lib().tsg_go_sort_perm(C.c_void_p(blob.ctypes.data),
                                     offs.ctypes.data_as(C.POINTER(C.c_uint64)),
                                     None if sec is None else sec.ctypes.data_as(C.POINTER(C.c_int64)),
                                     n, perm.ctypes.data_as(C.POINTER(C.c_uint32))))
    items[:] = [items[int(i)] for i in perm]


def sort_secrets(secrets):
    """AnalysisResult.Sort, secrets part (analyzer.go:212-223): files by FilePath, then each
    file's findings by (RuleID, StartLine), both with Go's unstable sort.Slice."""
    _go_sort(secrets, lambda s: s["FilePath"].encode("utf-8", "surrogateescape"))
    for s in secrets:
        _go_sort(s["Findings"], lambda f: f["RuleID"].encode("utf-8", "surrogateescape"),
                 lambda f: f["StartLine"])
    return secrets
