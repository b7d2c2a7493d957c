"""Image-layer ingest for the secret path: trivy's layer tar walker
(pkg/fanal/walker/tar.go, walk.go) feeding the batched analyzer.

  LayerTar(skip_files, skip_dirs).Walk(layer, fn)   walker/tar.go:33-84
  NativeLayer(scanner, tar_bytes, ...)             the same walk + Required + IsBinary in C++
                                                    (tsg_layer_pack), packed into one batch
  analyze_layer(analyzer, layer, ...)               walker.Walk + AnalyzerGroup.AnalyzeFile
                                                    (analyzer.go:395-445) + SecretAnalyzer,
                                                    with the files of a layer packed into
                                                    large batches for the MI355X kernels

The reference hands each file to a goroutine (≤5 per layer, image.go:28) that scans it
alone.  Here every file that passes `Required` is copied once into a batch; a batch of
`batch_bytes` is scanned in one call.  Per-file semantics are unchanged: the path passed
to `Required` is the cleaned tar name, the path given to `Scan` gets the "/" prefix of
image files (secret.go:90-96), and `IsBinary` uses the header size (secret.go:80).

Go's path helpers (filepath.Clean / Split / Join / Rel / Base on "/" paths) are restated
below because Python's posixpath differs on "//" prefixes, empty paths and "..".
"""
import ctypes as C
import tarfile

import numpy as np

from . import _native as N
from .analyzer import AnalysisInput, IsBinary, sort_secrets
from . import secret as S

OPQ = ".wh..wh..opq"   # tar.go:19
WH = ".wh."            # tar.go:20
APP_DIRS = [".git"]                 # walk.go:14
SYSTEM_DIRS = ["proc", "sys", "dev"]  # walk.go:15
THRESHOLD_SIZE = 200 << 20          # walk.go:18 (temp-file spill; no effect on results)

_REG = (tarfile.REGTYPE, tarfile.AREGTYPE)  # Go's reader maps TypeRegA to TypeReg


def clean(p):
    """Go path.Clean (lexical)."""
    if p == "":
        return "."
    rooted = p[0] == "/"
    out = []
    for part in p.split("/"):
        if part == "" or part == ".":
            continue
        if part == "..":
            if out and out[-1] != "..":
                out.pop()
            elif not rooted:
                out.append("..")
            continue
        out.append(part)
    s = "/".join(out)
    if rooted:
        return "/" + s
    return s or "."


def split(p):
    """Go filepath.Split: dir keeps its trailing slash."""
    i = p.rfind("/")
    return p[:i + 1], p[i + 1:]


def join(*elems):
    """Go filepath.Join: empty elements are ignored, the result is cleaned."""
    parts = [e for e in elems if e != ""]
    return clean("/".join(parts)) if parts else ""


def base(p):
    """Go filepath.Base."""
    if p == "":
        return "."
    p = p.rstrip("/")
    if p == "":
        return "/"
    return p[p.rfind("/") + 1:]


def rel(basepath, targpath):
    """Go filepath.Rel on "/" paths; returns None where Go returns an error."""
    b = clean(basepath)
    t = clean(targpath)
    if t == b:
        return "."
    if b == ".":
        b = ""
    if (len(b) > 0 and b[0] == "/") != (len(t) > 0 and t[0] == "/"):
        return None
    bl, tl = len(b), len(t)
    b0 = bi = t0 = ti = 0
    while True:
        while bi < bl and b[bi] != "/":
            bi += 1
        while ti < tl and t[ti] != "/":
            ti += 1
        if t[t0:ti] != b[b0:bi]:
            break
        if bi < bl:
            bi += 1
        if ti < tl:
            ti += 1
        b0, t0 = bi, ti
    if b[b0:bi] == "..":
        return None
    if b0 != bl:
        seps = b[b0:bl].count("/")
        s = ".." + "/.." * seps
        if t0 != tl:
            s += "/" + t[t0:]
        return s
    return t[t0:]


def under_skipped_dir(file_path, skip_dirs):
    """tar.go:100-111 (an error from Rel ends the search with False, as in Go)."""
    for sd in skip_dirs:
        r = rel(sd, file_path)
        if r is None:
            return False
        if not r.startswith("../"):
            return True
    return False


class LayerTar:
    """walker.LayerTar (tar.go:23-31, walk.go:25-76)."""

    def __init__(self, skip_files=(), skip_dirs=()):
        self.skip_files = [clean(f).lstrip("/") for f in skip_files]
        self.skip_dirs = [clean(d).lstrip("/") for d in list(skip_dirs) + SYSTEM_DIRS]

    def should_skip_file(self, p):
        return p.lstrip("/") in self.skip_files          # walk.go:48-54

    def should_skip_dir(self, d):
        d = d.lstrip("/")                                # walk.go:56-71
        return base(d) in APP_DIRS or d in self.skip_dirs

    def Walk(self, layer, fn):
        """tar.go:33-84.  `layer` is a binary file object (read sequentially).
        fn(file_path, size, read) is called for each regular file that is kept;
        `read()` returns its content.  Returns (opq_dirs, wh_files)."""
        opq_dirs, wh_files, skip_dirs = [], [], []
        with tarfile.open(fileobj=layer, mode="r|", encoding="utf-8",
                          errors="surrogateescape") as tr:
            for hdr in tr:
                file_path = clean(hdr.name).lstrip("/")
                file_dir, file_name = split(file_path)
                if file_name == OPQ:
                    opq_dirs.append(file_dir)
                    continue
                if file_name.startswith(WH):
                    wh_files.append(join(file_dir, file_name[len(WH):]))
                    continue
                if hdr.type == tarfile.DIRTYPE:
                    if self.should_skip_dir(file_path):
                        skip_dirs.append(file_path)
                        continue
                elif hdr.type in _REG:
                    if self.should_skip_file(file_path):
                        continue
                else:
                    continue  # links, devices, fifos, sparse/contiguous: no content
                if under_skipped_dir(file_path, skip_dirs):
                    continue
                if hdr.type == tarfile.DIRTYPE:
                    continue  # AnalyzeFile returns early for directories (analyzer.go:395)
                fn(file_path, hdr.size, lambda h=hdr: tr.extractfile(h).read())
        return opq_dirs, wh_files


def analyze_layer(analyzer, layer, device=None, ctx=None, emulate_chunk=0,
                  batch_bytes=1 << 30, skip_files=(), skip_dirs=()):
    """Secrets of one image layer: (sorted AnalysisResult.Secrets, opq_dirs, wh_files).

    Files are gated by `Required` on the cleaned path (analyzer.go:400-409) and by
    `IsBinary` on the header size, then packed into batches of about `batch_bytes` and
    scanned together (device/ctx: MI355X; emulate_chunk: kernel emulation; else the
    exact CPU batch path)."""
    scanner = analyzer.scanner
    secrets = []
    pending, pending_bytes = [], 0

    def flush():
        nonlocal pending, pending_bytes
        if pending:
            res = scanner.ScanBatch(pending, device=device, ctx=ctx, emulate_chunk=emulate_chunk)
            secrets.extend(r for r in res if r["Findings"])
        pending, pending_bytes = [], 0

    def on_file(file_path, size, read):
        nonlocal pending_bytes
        clean_path = file_path.lstrip("/")
        if not analyzer.Required(clean_path, size):
            return
        content = read()
        if IsBinary(content, size):
            return
        inp = AnalysisInput("", file_path, content)
        pending.append(S.ScanArgs(analyzer._scan_path(inp), content))
        pending_bytes += len(content)
        if pending_bytes >= batch_bytes:
            flush()

    opq, wh = LayerTar(skip_files, skip_dirs).Walk(layer, on_file)
    flush()
    return sort_secrets(secrets), opq, wh


class NativeLayer:
    """tsg_layer_pack: the walk, `Required` and `IsBinary` of a whole in-memory layer tar in
    one native pass; `.batch` views the packed files without a copy (valid while this
    object lives).  `.opq` / `.wh` are the walker's opaque dirs and whiteout files.  With
    world > 1 the batch holds only rank's contiguous byte run of the walked files
    (tsg_layer_pack_shard); opq / wh / walked are the whole layer's."""

    def __init__(self, scanner, tar, skip_files=(), skip_dirs=(), config_path="", rank=0, world=1):
        L = N.lib()
        self._h = None
        self._tar = np.frombuffer(tar, dtype=np.uint8) if len(tar) else np.zeros(1, np.uint8)
        enc = lambda xs: (C.c_char_p * max(1, len(xs)))(
            *[x.encode("utf-8", "surrogateescape") for x in xs])
        sf, sd = enc(list(skip_files)), enc(list(skip_dirs))
        h = C.c_void_p()
        # rank/world: tsg_layer_pack_shard, this rank's contiguous byte run of the layer
        N.check(L.tsg_layer_pack_shard(scanner.handle, C.c_void_p(self._tar.ctypes.data), len(tar),
                                       sf, len(skip_files), sd, len(skip_dirs),
                                       config_path.encode("utf-8", "surrogateescape"), rank, world,
                                       C.byref(h)))
        self._adopt(h)

    def _adopt(self, h):
        """Take ownership of a tsg_layer handle and view its batch, opq, wh and walked."""
        L = N.lib()
        self._h = h
        v = N.LayerView()
        N.check(L.tsg_layer_get(h, C.byref(v)))
        n = v.nfiles
        as_u64 = lambda p: np.ctypeslib.as_array(p, shape=(n + 1,))
        offs, poffs = as_u64(v.offsets), as_u64(v.path_offsets)
        as_u8 = lambda p, k: (np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(k,))
                              if p and k else np.zeros(1, np.uint8))
        self.batch = S.Batch(as_u8(v.data, int(offs[-1])), offs, as_u8(v.paths, int(poffs[-1])),
                             poffs)
        self.batch._owner = self
        self.opq = _nul_list(v.opq, v.opq_len)
        self.wh = _nul_list(v.wh, v.wh_len)
        self.walked = v.walked

    def __del__(self):
        if getattr(self, "_h", None):
            N.lib().tsg_layer_free(self._h)
            self._h = None


def _nul_list(p, k):
    return [x.decode("utf-8", "surrogateescape") for x in C.string_at(p, k).split(b"\0")[:-1]] if k else []


def _cstrs(xs):
    return (C.c_char_p * max(1, len(xs)))(*[x.encode("utf-8", "surrogateescape") for x in xs])


_NO_POS = (1 << 64) - 1


class LayerRange:
    """One rank's byte range of a layer's header chain (tsg_layer_range_*, trivy_secret.h):
    the speculative walk on construction (`.info` = lo, hi, start, end), then `sync(pos)`
    once the true chain's entry position is known, `dirs()` for the skip dirs it hands to
    later ranks, and `pack()` for its batch."""

    def __init__(self, tar, rank, world):
        L = N.lib()
        self._h = None
        self._tar = np.frombuffer(tar, dtype=np.uint8) if len(tar) else np.zeros(1, np.uint8)
        h, info = C.c_void_p(), (C.c_uint64 * 4)()
        N.check(L.tsg_layer_range_walk(C.c_void_p(self._tar.ctypes.data), len(tar), rank, world,
                                       C.byref(h), info))
        self._h = h
        self.info = tuple(int(x) for x in info)

    def sync(self, pos):
        end = C.c_uint64()
        N.check(N.lib().tsg_layer_range_sync(self._h, pos, C.byref(end)))
        return int(end.value)

    def dirs(self, skip_dirs=()):
        p, k = C.c_void_p(), C.c_uint64()
        N.check(N.lib().tsg_layer_range_dirs(self._h, _cstrs(list(skip_dirs)), len(skip_dirs),
                                             C.byref(p), C.byref(k)))
        return _nul_list(p.value, k.value)

    def pack(self, scanner, skip_files=(), skip_dirs=(), prior_dirs=(), config_path=""):
        h = C.c_void_p()
        N.check(N.lib().tsg_layer_range_pack(
            scanner.handle, self._h, _cstrs(list(skip_files)), len(skip_files),
            _cstrs(list(skip_dirs)), len(skip_dirs), _cstrs(list(prior_dirs)), len(prior_dirs),
            config_path.encode("utf-8", "surrogateescape"), C.byref(h)))
        lay = NativeLayer.__new__(NativeLayer)
        lay._tar = self._tar
        lay._range = self  # the entries' names live in the range; the batch copies the bytes
        lay._adopt(h)
        return lay

    def __del__(self):
        if getattr(self, "_h", None):
            N.lib().tsg_layer_range_free(self._h)
            self._h = None


def layer_chain_step(infos, confirmed):
    """The true header chain over ranks' ranges, as far as the exchanged data fixes it.

    infos[r] = LayerRange.info of rank r; confirmed[r] = the end rank r reported after
    tsg_layer_range_sync.  Returns ("done", pos) with every rank's entry position, or
    ("need", r, pos): rank r must sync at pos and publish its end (its speculative start
    was not on the chain, or the chain errs in its range)."""
    pos, out = 0, []
    for r, (lo, hi, start, end) in enumerate(infos):
        out.append(pos)
        if r in confirmed:
            pos = confirmed[r]
        elif pos >= hi:
            pass  # a member spans the range, or the archive ended before it
        elif start == pos and end != _NO_POS:
            pos = end  # a walk from a group position is deterministic
        else:
            return ("need", r, pos)
    return ("done", out)


def layer_chain(rng, rank, world, allgather, infos=None):
    """Fix the true chain across ranks (allgather(obj) -> list over ranks) and sync `rng` to
    it; returns this rank's entry position.  Raises the archive error of the chain on every
    rank, as one sequential walk fails.  infos: every rank's rng.info, when already gathered."""
    if infos is None:
        infos = allgather(rng.info)
    confirmed = {}
    while True:
        st = layer_chain_step(infos, confirmed)
        if st[0] == "done":
            pos = st[1][rank]
            rng.sync(pos)
            return pos
        _, r, pos = st
        msg = None
        if r == rank:
            try:
                msg = ("ok", rng.sync(pos))
            except Exception as e:  # noqa: BLE001 - forwarded to every rank
                msg = ("err", str(e))
        got = allgather(msg)[r]
        if got[0] == "err":
            raise RuntimeError(got[1])
        confirmed[r] = got[1]


def pack_layer_ranges(scanner, tar, world, skip_files=(), skip_dirs=(), config_path=""):
    """All `world` ranges of one layer in this process (the single-host form of the
    distributed index, and its test): returns the per-rank NativeLayer list."""
    rngs = [LayerRange(tar, r, world) for r in range(world)]
    infos = [g.info for g in rngs]
    confirmed = {}
    while True:
        st = layer_chain_step(infos, confirmed)
        if st[0] == "done":
            break
        _, r, pos = st
        confirmed[r] = rngs[r].sync(pos)
    for g, pos in zip(rngs, st[1]):
        g.sync(pos)
    dirs = [g.dirs(skip_dirs) for g in rngs]
    out, prior = [], []
    for r, g in enumerate(rngs):
        out.append(g.pack(scanner, skip_files, skip_dirs, prior, config_path))
        prior = prior + dirs[r]
    return out


class NativeFS(NativeLayer):
    """tsg_fs_pack: walker.FS.Walk + the fs artifact's relative paths + `Required` +
    `IsBinary` over a directory tree, files read in parallel and packed in path order
    (world > 1: tsg_fs_pack_shard, only this rank's contiguous byte run is read)."""

    def __init__(self, scanner, root, skip_files=(), skip_dirs=(), config_path="", rank=0, world=1):
        L = N.lib()
        self._h = None
        enc = lambda xs: (C.c_char_p * max(1, len(xs)))(
            *[x.encode("utf-8", "surrogateescape") for x in xs])
        sf, sd = enc(list(skip_files)), enc(list(skip_dirs))
        h = C.c_void_p()
        if world > 1:  # tsg_fs_pack_shard: this rank's contiguous byte run of the tree
            N.check(L.tsg_fs_pack_shard(scanner.handle, root.encode("utf-8", "surrogateescape"), sf,
                                        len(skip_files), sd, len(skip_dirs),
                                        config_path.encode("utf-8", "surrogateescape"), rank, world,
                                        C.byref(h)))
        else:
            N.check(L.tsg_fs_pack(scanner.handle, root.encode("utf-8", "surrogateescape"), sf,
                                  len(skip_files), sd, len(skip_dirs),
                                  config_path.encode("utf-8", "surrogateescape"), C.byref(h)))
        self._h = h
        v = N.LayerView()
        N.check(L.tsg_layer_get(h, C.byref(v)))
        n = v.nfiles
        as_u64 = lambda p: np.ctypeslib.as_array(p, shape=(n + 1,))
        offs, poffs = as_u64(v.offsets), as_u64(v.path_offsets)
        as_u8 = lambda p, k: (np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(k,))
                              if p and k else np.zeros(1, np.uint8))
        self.batch = S.Batch(as_u8(v.data, int(offs[-1])), offs, as_u8(v.paths, int(poffs[-1])),
                             poffs)
        self.batch._owner = self
        self.opq, self.wh = [], []
        self.walked = v.walked


class SlotIngest(NativeLayer):
    """Ingest straight into a pinned slot of a GpuContext (tsg_layer_pack_slot /
    tsg_fs_pack_slot / tsg_layer_range_pack_slot): the kept files are written once into the
    memory the device uploads from.  `.batch` views the slot; `scan()` submits it and returns
    the per-file results; `release()` (or garbage collection) gives the slot back."""

    @classmethod
    def layer(cls, ctx, tar, skip_files=(), skip_dirs=(), config_path=""):
        self = cls.__new__(cls)
        self._init(ctx, tar)
        h, sid = C.c_void_p(), C.c_uint32()
        N.check(N.lib().tsg_layer_pack_slot(ctx.handle, C.c_void_p(self._tar.ctypes.data), len(tar),
                                            _cstrs(list(skip_files)), len(skip_files),
                                            _cstrs(list(skip_dirs)), len(skip_dirs),
                                            config_path.encode("utf-8", "surrogateescape"),
                                            C.byref(sid), C.byref(h)))
        self._adopt_slot(h, sid.value)
        return self

    @classmethod
    def fs(cls, ctx, root, skip_files=(), skip_dirs=(), config_path=""):
        self = cls.__new__(cls)
        self._init(ctx, b"")
        h, sid = C.c_void_p(), C.c_uint32()
        N.check(N.lib().tsg_fs_pack_slot(ctx.handle, root.encode("utf-8", "surrogateescape"),
                                         _cstrs(list(skip_files)), len(skip_files),
                                         _cstrs(list(skip_dirs)), len(skip_dirs),
                                         config_path.encode("utf-8", "surrogateescape"),
                                         C.byref(sid), C.byref(h)))
        self._adopt_slot(h, sid.value)
        return self

    @classmethod
    def layer_range(cls, ctx, rng, skip_files=(), skip_dirs=(), prior_dirs=(), config_path=""):
        self = cls.__new__(cls)
        self._init(ctx, b"")
        self._tar, self._range = rng._tar, rng
        h, sid = C.c_void_p(), C.c_uint32()
        N.check(N.lib().tsg_layer_range_pack_slot(
            ctx.handle, rng._h, _cstrs(list(skip_files)), len(skip_files),
            _cstrs(list(skip_dirs)), len(skip_dirs), _cstrs(list(prior_dirs)), len(prior_dirs),
            config_path.encode("utf-8", "surrogateescape"), C.byref(sid), C.byref(h)))
        self._adopt_slot(h, sid.value)
        return self

    def _init(self, ctx, tar):
        self._h = None
        self._slot = None
        self._ctx = ctx
        self._tar = np.frombuffer(tar, dtype=np.uint8) if len(tar) else np.zeros(1, np.uint8)

    def _adopt_slot(self, h, sid):
        self._slot = sid
        self._adopt(h)

    def submit(self):
        """tsg_slot_submit of the packed files; the ticket (GpuContext.collect)."""
        return self._ctx.submit_slot(self._slot, self.batch.nfiles, self.batch)

    def scan(self):
        """Scan.Scan of every packed file, in batch order."""
        if not self.batch.nfiles:
            return []
        return self._ctx.collect(self.submit())

    def release(self):
        if self._slot is not None and self._ctx is not None and self._ctx.handle:
            self._ctx.release_slot(self._slot)
        self._slot = None

    def __del__(self):
        self.release()
        NativeLayer.__del__(self)


def scan_layer_pipelined(ctx, tar, skip_files=(), skip_dirs=(), config_path=""):
    """tsg_layer_scan: walk, gate and scan a layer in one pipelined call.  Returns
    (paths, per-file Scan results in that order, opq, wh, walked)."""
    t = np.frombuffer(tar, dtype=np.uint8) if len(tar) else np.zeros(1, np.uint8)
    h, out = C.c_void_p(), C.c_void_p()
    N.check(N.lib().tsg_layer_scan(ctx.handle, C.c_void_p(t.ctypes.data), len(tar),
                                   _cstrs(list(skip_files)), len(skip_files),
                                   _cstrs(list(skip_dirs)), len(skip_dirs),
                                   config_path.encode("utf-8", "surrogateescape"),
                                   C.byref(h), C.byref(out)))
    return _pipelined_result(ctx, h, out)


def scan_fs_pipelined(ctx, root, skip_files=(), skip_dirs=(), config_path=""):
    """tsg_fs_scan: walk, gate and scan a tree in one pipelined call."""
    h, out = C.c_void_p(), C.c_void_p()
    N.check(N.lib().tsg_fs_scan(ctx.handle, root.encode("utf-8", "surrogateescape"),
                                _cstrs(list(skip_files)), len(skip_files),
                                _cstrs(list(skip_dirs)), len(skip_dirs),
                                config_path.encode("utf-8", "surrogateescape"),
                                C.byref(h), C.byref(out)))
    return _pipelined_result(ctx, h, out)


def _pipelined_result(ctx, h, out):
    L = N.lib()
    try:
        v = N.LayerView()
        N.check(L.tsg_layer_get(h, C.byref(v)))
        n = v.nfiles
        poffs = np.ctypeslib.as_array(v.path_offsets, shape=(n + 1,))
        raw = C.string_at(v.paths, int(poffs[-1])) if n and poffs[-1] else b""
        paths = [raw[int(poffs[i]):int(poffs[i + 1])].decode("utf-8", "surrogateescape") for i in range(n)]
        opq, wh, walked = _nul_list(v.opq, v.opq_len), _nul_list(v.wh, v.wh_len), v.walked
    finally:
        L.tsg_layer_free(h)
    return paths, ctx.scanner.decode(out, paths), opq, wh, walked


def analyze_fs(analyzer, root, device=None, ctx=None, emulate_chunk=0, skip_files=(), skip_dirs=()):
    """`trivy fs --security-checks secret <root>`'s secret analysis (BASELINE configs[0]):
    the native fs ingest, one batch, the sorted AnalysisResult.Secrets."""
    fs = NativeFS(analyzer.scanner, root, skip_files, skip_dirs, analyzer.configPath)
    res = analyzer.scanner.ScanBatch(fs.batch, device=device, ctx=ctx,
                                     emulate_chunk=emulate_chunk) if fs.batch.nfiles else []
    return sort_secrets([r for r in res if r["Findings"]])


def analyze_layer_native(analyzer, tar, device=None, ctx=None, emulate_chunk=0,
                         skip_files=(), skip_dirs=()):
    """analyze_layer over an in-memory tar with the native ingest (one batch per layer)."""
    lay = NativeLayer(analyzer.scanner, tar, skip_files, skip_dirs, analyzer.configPath)
    res = analyzer.scanner.ScanBatch(lay.batch, device=device, ctx=ctx,
                                     emulate_chunk=emulate_chunk) if lay.batch.nfiles else []
    return sort_secrets([r for r in res if r["Findings"]]), lay.opq, lay.wh
