"""Host-side mirror of trivy's `pkg/fanal/secret` API over the native engine.

Same names, argument meaning and error behaviour as the reference:
  Config / Rule / AllowRule / ExcludeBlock / Global      scanner.go:23-94, 186-225
  ParseConfig(path) -> Config | None                      scanner.go:267-291
  NewScanner(config) -> Scanner                           scanner.go:293-329
  Scanner.Scan(ScanArgs) -> Secret                        scanner.go:341-416 (exact, CPU)
  Scanner.AllowPath(path)                                 scanner.go:55-57
and the batching boundary the GPU needs:
  Scanner.ScanBatch([ScanArgs], device=...) -> [Secret]   (K1 + K2 on the MI355X, exact
                                                          host resolution of candidates)

`Secret` values are dicts shaped like Go's types.Secret:
  {"FilePath": str, "Findings": None | [SecretFinding]}
with SecretFinding = {"RuleID", "Category", "Severity", "Title", "StartLine", "EndLine",
"Code": {"Lines": [Line]}, "Match"}; Match and line Content/Highlighted are `bytes`
(Go strings are byte strings; content need not be valid UTF-8).
"""
import ctypes as C
import json
import os
import struct
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import yaml

from . import _native as N

_RULES_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rules",
                           "builtin_rules.json")


class ConfigError(ValueError):
    """secrets config decode / regexp compile error (scanner.go:74-77, 286-288)."""


def _check_regex(src):
    """regexp.Compile on the native engine; raises ConfigError like UnmarshalYAML."""
    h = C.c_void_p()
    err = C.create_string_buffer(512)
    rc = N.lib().tsg_regex_compile(src.encode("utf-8", "surrogateescape"), C.byref(h), err, 512)
    if rc != N.TSG_OK:
        raise ConfigError("regexp compile error: %s" % err.value.decode("utf-8", "replace"))
    N.lib().tsg_regex_free(h)
    return src


@dataclass
class AllowRule:
    ID: str = ""
    Description: str = ""
    Regex: Optional[str] = None
    Path: Optional[str] = None


@dataclass
class ExcludeBlock:
    Description: str = ""
    Regexes: List[str] = field(default_factory=list)


@dataclass
class Rule:
    ID: str = ""
    Category: str = ""
    Title: str = ""
    Severity: str = ""
    Regex: Optional[str] = None
    Keywords: List[str] = field(default_factory=list)
    Path: Optional[str] = None
    AllowRules: List[AllowRule] = field(default_factory=list)
    ExcludeBlock: ExcludeBlock = field(default_factory=ExcludeBlock)
    SecretGroupName: str = ""


@dataclass
class Config:
    EnableBuiltinRuleIDs: List[str] = field(default_factory=list)
    DisableRuleIDs: List[str] = field(default_factory=list)
    DisableAllowRuleIDs: List[str] = field(default_factory=list)
    CustomRules: List[Rule] = field(default_factory=list)
    CustomAllowRules: List[AllowRule] = field(default_factory=list)
    ExcludeBlock: ExcludeBlock = field(default_factory=ExcludeBlock)


@dataclass
class ScanArgs:
    FilePath: str
    Content: bytes


def _s(v):
    return "" if v is None else str(v)


def _rx(v):
    return None if v is None else _check_regex(str(v))


def _allow(lst):
    return [AllowRule(_s(a.get("id")), _s(a.get("description")), _rx(a.get("regex")),
                      _rx(a.get("path"))) for a in (lst or [])]


def _exclude(d):
    d = d or {}
    return ExcludeBlock(_s(d.get("description")), [_rx(x) for x in (d.get("regexes") or [])])


def config_from_dict(doc):
    if not isinstance(doc, dict):
        raise ConfigError("secrets config decode error")
    c = Config()
    c.EnableBuiltinRuleIDs = [str(x) for x in (doc.get("enable-builtin-rules") or [])]
    c.DisableRuleIDs = [str(x) for x in (doc.get("disable-rules") or [])]
    c.DisableAllowRuleIDs = [str(x) for x in (doc.get("disable-allow-rules") or [])]
    for r in doc.get("rules") or []:
        c.CustomRules.append(Rule(
            ID=_s(r.get("id")), Category=_s(r.get("category")), Title=_s(r.get("title")),
            Severity=_s(r.get("severity")), Regex=_rx(r.get("regex")),
            Keywords=[str(k) for k in (r.get("keywords") or [])], Path=_rx(r.get("path")),
            AllowRules=_allow(r.get("allow-rules")), ExcludeBlock=_exclude(r.get("exclude-block")),
            SecretGroupName=_s(r.get("secret-group-name"))))
    c.CustomAllowRules = _allow(doc.get("allow-rules"))
    c.ExcludeBlock = _exclude(doc.get("exclude-block"))
    return c


def ParseConfig(config_path):
    """scanner.go:267-291: "" or a missing file -> None (builtins only)."""
    if not config_path:
        return None
    if not os.path.exists(config_path):
        return None
    with open(config_path, "rb") as f:
        doc = yaml.safe_load(f)
    if doc is None:
        raise ConfigError("secrets config decode error: EOF")
    return config_from_dict(doc)


_BUILTINS = None


def builtin_rules():
    """The 83 builtin rules and 12 builtin allow rules (builtin-rules.go, builtin-allow-rules.go)."""
    global _BUILTINS
    if _BUILTINS is None:
        d = json.load(open(_RULES_JSON))
        rules = [Rule(ID=r["id"], Category=r["category"], Title=r["title"],
                      Severity=r["severity"], Regex=r["regex"], Keywords=list(r["keywords"]),
                      SecretGroupName=r["secret_group_name"]) for r in d["rules"]]
        allow = [AllowRule(a["id"], a["description"], a["regex"], a["path"])
                 for a in d["allow_rules"]]
        _BUILTINS = (rules, allow)
    return _BUILTINS


def NewScanner(config=None):
    """scanner.go:293-329"""
    b_rules, b_allow = builtin_rules()
    if config is None:
        return Scanner(list(b_rules), list(b_allow), ExcludeBlock())
    enabled = list(b_rules)
    if config.EnableBuiltinRuleIDs:
        enabled = [r for r in b_rules if r.ID in config.EnableBuiltinRuleIDs]
    enabled = enabled + list(config.CustomRules)
    rules = [r for r in enabled if r.ID not in config.DisableRuleIDs]
    allow = [a for a in list(b_allow) + list(config.CustomAllowRules)
             if a.ID not in config.DisableAllowRuleIDs]
    return Scanner(rules, allow, config.ExcludeBlock)


def _b(s):
    return None if s is None else s.encode("utf-8", "surrogateescape")


class _Keep:
    """Keeps ctypes buffers alive for the duration of a native call."""

    def __init__(self):
        self.refs = []

    def cstr(self, s):
        b = _b(s)
        self.refs.append(b)
        return b

    def arr(self, ctype, items):
        a = (ctype * max(1, len(items)))(*items)
        self.refs.append(a)
        return a


class Batch:
    """Files packed for the engine: one contiguous byte stream + u64 offsets (+ paths)."""

    def __init__(self, data, offsets, paths, path_offsets):
        self.data = np.ascontiguousarray(data, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.paths = np.ascontiguousarray(paths, dtype=np.uint8)
        self.path_offsets = np.ascontiguousarray(path_offsets, dtype=np.uint64)
        self.nfiles = len(self.offsets) - 1

    @classmethod
    def from_args(cls, args):
        lens = np.array([len(a.Content) for a in args], dtype=np.uint64)
        offs = np.zeros(len(args) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        data = np.frombuffer(b"".join(a.Content for a in args) or b"\0", dtype=np.uint8)
        pb = [a.FilePath.encode("utf-8", "surrogateescape") for a in args]
        plens = np.array([len(p) for p in pb], dtype=np.uint64)
        poffs = np.zeros(len(args) + 1, dtype=np.uint64)
        np.cumsum(plens, out=poffs[1:])
        paths = np.frombuffer(b"".join(pb) or b"\0", dtype=np.uint8)
        return cls(data, offs, paths, poffs)

    def ptrs(self):
        u64p = C.POINTER(C.c_uint64)
        return (C.c_void_p(self.data.ctypes.data), self.offsets.ctypes.data_as(u64p),
                C.c_uint32(self.nfiles), C.c_void_p(self.paths.ctypes.data),
                self.path_offsets.ctypes.data_as(u64p))

    def path(self, i):
        return bytes(self.paths[int(self.path_offsets[i]):int(self.path_offsets[i + 1])]).decode(
            "utf-8", "surrogateescape")


class Scanner:
    """secret.Scanner{Global}: compiled once, shared read-only (thread-safe natively)."""

    def __init__(self, rules, allow_rules, exclude_block):
        self.Rules = list(rules)
        self.AllowRules = list(allow_rules)
        self.ExcludeBlock = exclude_block
        self._h = None
        self._compile()

    def _compile(self):
        L = N.lib()
        keep = _Keep()
        descs = []
        for r in self.Rules:
            kws = keep.arr(C.c_char_p, [keep.cstr(k) for k in r.Keywords])
            ars = keep.arr(N.AllowRuleDesc, [N.AllowRuleDesc(keep.cstr(a.ID),
                                                              keep.cstr(a.Description),
                                                              keep.cstr(a.Regex), keep.cstr(a.Path))
                                              for a in r.AllowRules])
            exc = keep.arr(C.c_char_p, [keep.cstr(x) for x in r.ExcludeBlock.Regexes])
            descs.append(N.RuleDesc(keep.cstr(r.ID), keep.cstr(r.Category), keep.cstr(r.Title),
                                    keep.cstr(r.Severity), keep.cstr(r.Regex), kws,
                                    len(r.Keywords), keep.cstr(r.Path), ars, len(r.AllowRules),
                                    exc, len(r.ExcludeBlock.Regexes),
                                    keep.cstr(r.SecretGroupName)))
        rd = keep.arr(N.RuleDesc, descs)
        ad = keep.arr(N.AllowRuleDesc, [N.AllowRuleDesc(keep.cstr(a.ID), keep.cstr(a.Description),
                                                        keep.cstr(a.Regex), keep.cstr(a.Path))
                                        for a in self.AllowRules])
        ex = keep.arr(C.c_char_p, [keep.cstr(x) for x in self.ExcludeBlock.Regexes])
        h = C.c_void_p()
        err = C.create_string_buffer(1024)
        rc = L.tsg_ruleset_compile(rd, len(descs), ad, len(self.AllowRules), ex,
                                   len(self.ExcludeBlock.Regexes), C.byref(h), err, 1024)
        if rc == N.TSG_ERR_CONFIG:
            raise ConfigError(err.value.decode("utf-8", "replace"))
        N.check(rc)
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            N.lib().tsg_ruleset_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def info(self):
        i = N.RulesetInfo()
        N.check(N.lib().tsg_ruleset_get_info(self._h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in N.RulesetInfo._fields_}

    def k1_reference(self, batch, chunk):
        """K1 semantics on the CPU (same layout as GpuContext.k1_output)."""
        import numpy as np
        W = (self.info()["n_keywords"] + 31) // 32
        kw = np.zeros(batch.nfiles * W, dtype=np.uint32)
        ev = np.zeros((int(batch.offsets[-1]) + chunk - 1) // chunk, dtype=np.uint32)
        u32p = C.POINTER(C.c_uint32)
        N.check(N.lib().tsg_emulate_k1(self.handle, C.c_void_p(batch.data.ctypes.data),
                                       batch.offsets.ctypes.data_as(C.POINTER(C.c_uint64)),
                                       batch.nfiles, chunk, kw.ctypes.data_as(u32p), kw.size,
                                       ev.ctypes.data_as(u32p), ev.size))
        return kw.reshape(batch.nfiles, W), ev

    def k1_literals(self):
        """K1's literals as (bytes, event bits); ids below n_keywords are keywords."""
        out = []
        buf = C.create_string_buffer(1 << 16)
        n, ev = C.c_uint32(), C.c_uint32()
        while N.lib().tsg_ruleset_k1_literal(self._h, len(out), buf, len(buf), C.byref(n), C.byref(ev)) == 0:
            out.append((buf.raw[:n.value], ev.value))
        return out

    def k1f_emulate(self, batch, chunk, quiet=(), sample_kib=0):
        """K1F's algorithm on the CPU (k1f.hpp): (keyword bits, chunk events, stats); with
        sample_kib the filter is priced on the batch's first sample_kib KiB."""
        import numpy as np
        W = (self.info()["n_keywords"] + 31) // 32
        kw = np.zeros(batch.nfiles * W, dtype=np.uint32)
        ev = np.zeros((int(batch.offsets[-1]) + chunk - 1) // chunk, dtype=np.uint32)
        q = np.array(list(quiet) or [0], dtype=np.uint32)
        st = np.zeros(4, dtype=np.uint64)
        u32p = C.POINTER(C.c_uint32)
        N.check(N.lib().tsg_emulate_k1f(self.handle, C.c_void_p(batch.data.ctypes.data),
                                        batch.offsets.ctypes.data_as(C.POINTER(C.c_uint64)),
                                        batch.nfiles, chunk, q.ctypes.data_as(u32p), len(quiet),
                                        sample_kib, kw.ctypes.data_as(u32p), kw.size, ev.ctypes.data_as(u32p),
                                        ev.size, st.ctypes.data_as(C.POINTER(C.c_uint64))))
        return kw.reshape(batch.nfiles, W), ev, {"groups": int(st[0]), "arrivals": int(st[1]),
                                                 "records": int(st[2])}

    def AllowPath(self, path):
        b = _b(path)
        rc = N.lib().tsg_ruleset_allow_path(self._h, b, len(b))
        if rc < 0:
            N.check(rc)
        return rc == 1

    def Scan(self, args):
        """scanner.go:341-416 on the exact CPU path."""
        p = _b(args.FilePath)
        out = C.c_void_p()
        N.check(N.lib().tsg_scan_cpu(self._h, p, len(p), bytes(args.Content), len(args.Content),
                                     C.byref(out)))
        return self.decode(out, [args.FilePath])[0]

    def ScanBatch(self, args, device=None, ctx=None, emulate_chunk=0, nthreads=0):
        """Scan many files.  device=int -> MI355X kernels; emulate_chunk>0 -> the kernels'
        algorithm emulated on the CPU (tests); otherwise the exact CPU batch path."""
        batch = args if isinstance(args, Batch) else Batch.from_args(args)
        paths = [batch.path(i) for i in range(batch.nfiles)]
        out = C.c_void_p()
        L = N.lib()
        if device is not None or ctx is not None:
            own = ctx is None
            if own:
                ctx = GpuContext(self, device)
            try:
                N.check(L.tsg_scan_batch(ctx.handle, *batch.ptrs(), C.byref(out)))
            finally:
                if own:
                    ctx.close()
        elif emulate_chunk:
            N.check(L.tsg_scan_batch_emulated(self._h, *batch.ptrs(), emulate_chunk, C.byref(out)))
        else:
            N.check(L.tsg_scan_cpu_batch(self._h, *batch.ptrs(), nthreads, C.byref(out)))
        return self.decode(out, paths)

    def decode(self, out, paths):
        L = N.lib()
        n = C.c_size_t()
        ptr = L.tsg_result_data(out, C.byref(n))
        buf = C.string_at(ptr, n.value)
        L.tsg_result_free(out)
        return decode_results(buf, paths, self.Rules)


def decode_results(buf, paths, rules):
    magic, nfiles = struct.unpack_from("<II", buf, 0)
    assert magic == 0x31475354 and nfiles == len(paths)
    pos = 8
    out = []
    for i in range(nfiles):
        status = buf[pos]
        (nf,) = struct.unpack_from("<I", buf, pos + 1)
        pos += 5
        findings = []
        for _ in range(nf):
            ri, sl, el, ml = struct.unpack_from("<IiiI", buf, pos)
            pos += 16
            match = buf[pos:pos + ml]
            pos += ml
            (nl,) = struct.unpack_from("<I", buf, pos)
            pos += 4
            lines = []
            for _ in range(nl):
                num, fl, cl = struct.unpack_from("<iBI", buf, pos)
                pos += 9
                content = buf[pos:pos + cl]
                pos += cl
                lines.append({"Number": num, "Content": content, "IsCause": bool(fl & 1),
                              "Annotation": "", "Truncated": False, "Highlighted": content,
                              "FirstCause": bool(fl & 2), "LastCause": bool(fl & 4)})
            r = rules[ri]
            findings.append({"RuleID": r.ID, "Category": r.Category,
                             "Severity": r.Severity if r.Severity != "" else "UNKNOWN",
                             "Title": r.Title, "StartLine": sl, "EndLine": el,
                             "Code": {"Lines": lines or None}, "Match": match})
        if status == 0:
            out.append({"FilePath": "", "Findings": None})
        elif status == 1:
            out.append({"FilePath": paths[i], "Findings": None})
        else:
            out.append({"FilePath": paths[i], "Findings": findings})
    return out


class GpuContext:
    """One device context (tsg_ctx): rule tables replicated in HBM, two lanes, pinned slots.

    upload() copies a batch into a pinned slot that this object then holds (the library
    keeps no pointer to the caller's buffers); submit() / submit_slot() return the native
    ticket of the submission and collect(ticket) decodes its results with the paths it was
    submitted with (collect() with no ticket takes this object's oldest submission).
    scan_batch() is the one-call, thread-safe Scan of a batch.  emulate=True runs the
    kernels' algorithm on the CPU over the same pipeline (tests without a GPU)."""

    def __init__(self, scanner, device=0, chunk_bytes=0, ext_cap=0, cand_capacity=0,
                 host_threads=0, adapt_mib=0, emulate=False, slot_mib=0, max_slots=0):
        import threading
        self._h = None
        self._owned = True
        self.scanner = scanner
        self.chunk = chunk_bytes or 256
        opt = N.CtxOptions(chunk_bytes, ext_cap, cand_capacity, host_threads, adapt_mib,
                           N.TSG_CTX_EMULATE if emulate else 0, slot_mib, max_slots)
        h = C.c_void_p()
        N.check(N.lib().tsg_ctx_create(int(device), scanner.handle, C.byref(opt), C.byref(h)))
        self._h = h
        self._upload = None     # (slot id, Batch) of the last upload
        self._k1 = None
        self._lock = threading.Lock()
        self._fifo = []         # (ticket, paths) of this object's uncollected submissions
        self._paths = {}        # ticket -> paths

    @classmethod
    def borrowed(cls, scanner, handle, chunk_bytes=0):
        """A view of a context owned elsewhere (a device of a MultiGpu): same methods, and
        close() leaves the context itself alone."""
        import threading
        self = cls.__new__(cls)
        self._h = handle
        self._owned = False
        self.scanner = scanner
        self.chunk = chunk_bytes or 256
        self._upload = None
        self._k1 = None
        self._lock = threading.Lock()
        self._fifo = []
        self._paths = {}
        return self

    @property
    def handle(self):
        return self._h

    def upload(self, batch):
        """Copy the batch into a pinned slot held by this object (the previous upload's slot
        is given back)."""
        sid = C.c_uint32()
        N.check(N.lib().tsg_batch_upload(self._h, *batch.ptrs(), C.byref(sid)))
        with self._lock:
            prev, self._upload = self._upload, (sid.value, batch)
        if prev is not None:
            N.check(N.lib().tsg_slot_release(self._h, prev[0]))

    def kernels(self):
        """The device part of a scan of the uploaded batch, synchronously (test hook);
        k1_output() then returns its keyword bits and chunk events."""
        sid, b = self._upload
        W = (self.scanner.info()["n_keywords"] + 31) // 32
        kw = np.zeros(b.nfiles * W, dtype=np.uint32)
        ev = np.zeros((int(b.offsets[-1]) + self.chunk - 1) // self.chunk, dtype=np.uint32)
        u32p = C.POINTER(C.c_uint32)
        N.check(N.lib().tsg_batch_kernels(self._h, sid, b.nfiles, kw.ctypes.data_as(u32p), kw.size,
                                          ev.ctypes.data_as(u32p), ev.size))
        self._k1 = (kw.reshape(b.nfiles, W), ev)

    def k1_output(self, chunk):
        """(keyword bits [nfiles, kw_words], chunk event bits) of the last kernels() call."""
        assert chunk == self.chunk, "the context's chunk is %d" % self.chunk
        return self._k1

    @staticmethod
    def _paths_of(batch):
        if isinstance(batch, Batch):
            return [batch.path(i) for i in range(batch.nfiles)]
        return list(batch)

    def _track(self, ticket, paths_of):
        with self._lock:
            self._fifo.append(ticket)
            self._paths[ticket] = paths_of
        return ticket

    def submit(self):
        """Device part of a scan of the uploaded batch, asynchronously; its host resolution
        follows it in the background.  Returns the ticket."""
        sid, b = self._upload
        t = C.c_uint64()
        N.check(N.lib().tsg_slot_submit(self._h, sid, b.nfiles, C.byref(t)))
        return self._track(t.value, b)

    def submit_slot(self, slot_id, nfiles, paths_of):
        """Submit the first nfiles files of an acquired slot (see acquire_slot); paths_of is
        the Batch or the list of paths they were packed from.  Returns the ticket."""
        if paths_of is None:
            raise ValueError("submit_slot needs the submitted files' paths (a Batch or a list)")
        t = C.c_uint64()
        N.check(N.lib().tsg_slot_submit(self._h, int(slot_id), int(nfiles), C.byref(t)))
        return self._track(t.value, paths_of)

    def acquire_slot(self, data_bytes, nfiles, path_bytes):
        """A pinned slot to fill directly: (id, data, offsets, paths, path_offsets) as
        numpy views of the library's pinned memory."""
        v = N.SlotView()
        N.check(N.lib().tsg_slot_acquire(self._h, int(data_bytes), int(nfiles),
                                         int(path_bytes), C.byref(v)))
        data = np.ctypeslib.as_array((C.c_uint8 * v.data_cap).from_address(v.data))
        offs = np.ctypeslib.as_array(v.offsets, shape=(v.files_cap + 1,))
        paths = np.ctypeslib.as_array((C.c_uint8 * v.paths_cap).from_address(v.paths))
        poffs = np.ctypeslib.as_array(v.path_offsets, shape=(v.files_cap + 1,))
        return v.id, data, offs, paths, poffs

    def release_slot(self, slot_id):
        N.check(N.lib().tsg_slot_release(self._h, int(slot_id)))

    def _take(self, ticket):
        with self._lock:
            if ticket is None:
                if not self._fifo:
                    raise N.NativeError(N.TSG_ERR_ARG, "no submitted batch")
                ticket = self._fifo.pop(0)
            elif ticket in self._paths:
                self._fifo.remove(ticket)
            return ticket, self._paths.pop(ticket, None)

    def collect_raw(self, ticket=None):
        """Results of one submission (default: this object's oldest) as a raw tsg_result
        handle; the caller frees it."""
        ticket, _ = self._take(ticket)
        out = C.c_void_p()
        N.check(N.lib().tsg_batch_collect(self._h, ticket, C.byref(out)))
        return out

    def collect(self, ticket=None):
        ticket, paths = self._take(ticket)
        out = C.c_void_p()
        N.check(N.lib().tsg_batch_collect(self._h, ticket, C.byref(out)))
        return self.scanner.decode(out, self._paths_of(paths))

    def pending(self):
        """Uncollected submissions of the context (every caller)."""
        return N.lib().tsg_batch_pending(self._h)

    def scan(self):
        return self.collect(self.submit())

    def scan_batch(self, batch):
        """tsg_scan_batch: copy, scan and resolve one batch in a slot of its own
        (thread-safe: any number of threads may call it on one context)."""
        out = C.c_void_p()
        N.check(N.lib().tsg_scan_batch(self._h, *batch.ptrs(), C.byref(out)))
        return self.scanner.decode(out, self._paths_of(batch))

    def stats(self):
        s = N.Stats()
        N.check(N.lib().tsg_ctx_get_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in N.Stats._fields_}

    def close(self):
        if self._h:
            if self._upload is not None:
                N.lib().tsg_slot_release(self._h, self._upload[0])
                self._upload = None
            if self._owned:
                N.lib().tsg_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class MultiGpu:
    """tsg_multi: one process driving several devices (trivy's per-layer goroutines over a
    node's GPUs, pkg/fanal/artifact/image/image.go:210-234).  scan_batch() shards a batch's
    files LPT by bytes over the devices and returns the results in input order."""

    def __init__(self, scanner, devices, slot_mib=0, host_threads=0, emulate=False, max_slots=0,
                 chunk_bytes=0):
        self._h = None
        self.scanner = scanner
        self.chunk = chunk_bytes or 256
        opt = N.CtxOptions(chunk_bytes, 0, 0, host_threads, 0, N.TSG_CTX_EMULATE if emulate else 0,
                           slot_mib, max_slots)
        devs = (C.c_int * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        N.check(N.lib().tsg_multi_create(devs, len(devices), scanner.handle, C.byref(opt),
                                         C.byref(h)))
        self._h = h
        self.n = len(devices)

    def scan_batch(self, batch):
        out = C.c_void_p()
        N.check(N.lib().tsg_multi_scan_batch(self._h, *batch.ptrs(), C.byref(out)))
        return self.scanner.decode(out, GpuContext._paths_of(batch))

    def context(self, i):
        """The i-th device's context (owned by this object) as a GpuContext view."""
        h = C.c_void_p()
        N.check(N.lib().tsg_multi_ctx(self._h, int(i), C.byref(h)))
        return GpuContext.borrowed(self.scanner, h, self.chunk)

    def stats(self, i):
        s = N.Stats()
        N.check(N.lib().tsg_multi_get_stats(self._h, int(i), C.byref(s)))
        return {k: getattr(s, k) for k, _ in N.Stats._fields_}

    def close(self):
        if self._h:
            N.lib().tsg_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class ScanQueue:
    """tsg_queue: Scan(ScanArgs) for many concurrent callers sharing one context; their
    files are coalesced into pinned batches (the analyzer's per-file goroutines,
    pkg/fanal/analyzer/analyzer.go:419-443)."""

    def __init__(self, ctx, flush_us=2000):
        self.ctx = ctx
        h = C.c_void_p()
        N.check(N.lib().tsg_queue_create(ctx.handle, int(flush_us), C.byref(h)))
        self._h = h

    def Scan(self, args):
        p = _b(args.FilePath)
        out = C.c_void_p()
        N.check(N.lib().tsg_queue_scan(self._h, p, len(p), bytes(args.Content),
                                       len(args.Content), C.byref(out)))
        return self.ctx.scanner.decode(out, [args.FilePath])[0]

    def flush(self):
        N.check(N.lib().tsg_queue_flush(self._h))

    def close(self):
        if self._h:
            N.lib().tsg_queue_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()
