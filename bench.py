#!/usr/bin/env python3
"""Secret-scan throughput on MI355X (BASELINE.json metric, configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--gb G]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

GPUs: under torchrun, one rank per GPU (rank r drives device LOCAL_RANK; WORLD_SIZE must
equal --gpus).  Without torchrun, --gpus N makes this one process drive devices 0..N-1
through tsg_multi (the form a single trivy process binds, image.go:210-234), one host
thread per device.  Fewer visible GPUs than asked is an error, never a silent fallback.

Workload (per GPU, weak scaling): the 83 builtin rules over a seeded synthetic corpus of
--gb GiB (default 10: BASELINE configs[1]) of mixed code/config text files with planted
secrets.  The corpus is packed once, before timing, into the context's pinned host slots
(--batch-mib each; the ingest of SURVEY.md §8f writes files straight into such slots).
One step = one scan of the whole corpus from host memory: for every slot, H2D into HBM,
K1 keyword automaton, gates, device-side item layout, K2 rule-group DFAs, outputs back to
pinned host memory, then exact host resolution of every finding (Go semantics) and
serialization of every per-file result.  Batches are pipelined across two device lanes
(the H2D of one overlaps the kernels of the other) and --depth batches in flight; every
byte crosses PCIe in every step.  value = content bytes of all ranks x steps / max-over-
ranks wall time of the timed steps.

Rank 0 prints ONE JSON line with, besides the contract fields:
  roofline       K1 (the dominant kernel): algorithmic bytes per launch / mean HIP-event
                 duration of its launches (events on the lane stream around each launch)
                 vs 8 TB/s; traffic = HBM bytes per launch from the FETCH_SIZE pass of the
                 same command recorded in profiles/pmc/<rules>.json, used only when that
                 pass ran the same device code (sha256 of the HIP sources) and batch size,
                 else null; converted with the factor calibrated for K1's access pattern
                 (tools/fetch_calib.hip)
  kernels        K1, K2 (on the bytes it reads) and K1+gates+K2 GB/s (HIP events)
  pipeline       H2D GB/s, per-batch stage times, resolution time
  cpu_baseline   the library's exact C++ CPU path (the reference algorithm restated:
                 per-rule keyword gate on bytes.ToLower, Go-semantics regexp over whole
                 files) on this host's cores, on a bounded sample of the same corpus
  cpu_optimised  the GPU algorithm (K1 automaton + K2 DFAs + the same exact resolution)
                 emulated on the same cores and sample
  checks         every step's findings (files with findings, findings) must equal the
                 warmup step's, and a device scan of the cpu_baseline sample must be
                 byte-identical to the exact CPU path's result; the bench fails otherwise
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# FETCH_SIZE passes of this command per rule set (rocprofv3 --pmc FETCH_SIZE, recorded by
# tools/pmc_traffic.py --record), committed under profiles/
PMC_DIR = os.path.join(ROOT, "profiles", "pmc")


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return None, 0, 1, 0
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo")
    return dist, dist.get_rank(), ws, int(os.environ.get("LOCAL_RANK", "0"))


def _barrier(dist):
    """Barrier + device sync (every batch runs on the library's own lane streams and is
    collected inside the timed region; torch's synchronize covers anything else)."""
    if dist is not None:
        dist.barrier()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except ImportError:
        pass


def _reduce(dist, v, op):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
    return float(t.item())


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """The CPUs this process may use: the affinity mask, the cgroup's CPU quota (cpu.max) and
    the harness's thread budget (OMP_NUM_THREADS; 16 per GPU on the GPU box, where nproc
    counts the whole machine).  Returns (threads, details)."""
    det = {"nproc": os.cpu_count()}
    n = os.cpu_count() or 1
    try:
        det["affinity"] = len(os.sched_getaffinity(0))
        n = min(n, det["affinity"])
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            det["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        det["omp_num_threads"] = int(omp)
        n = min(n, int(omp))
    det["threads_used"] = n
    return n, det


def _sub_batch(batch, max_bytes):
    from trivy_amd.secret import Batch
    nf = 0
    while nf < batch.nfiles and int(batch.offsets[nf + 1]) <= max_bytes:
        nf += 1
    nf = max(nf, 1)
    return Batch(batch.data[:int(batch.offsets[nf])], batch.offsets[:nf + 1],
                 batch.paths[:int(batch.path_offsets[nf])], batch.path_offsets[:nf + 1]), nf


def cpu_baselines(sc, batch, max_bytes, nthreads):
    """The exact CPU path (the reference algorithm, restated in C++) and the optimised CPU
    path (the GPU algorithm emulated), both on `nthreads` threads over the same prefix.
    Returns them with the sample and the exact path's raw result bytes."""
    from trivy_amd import _native as N
    import ctypes as C
    L = N.lib()
    sub, nf = _sub_batch(batch, max_bytes)
    nb = int(sub.offsets[-1])
    out = C.c_void_p()
    t0 = time.perf_counter()
    N.check(L.tsg_scan_cpu_batch(sc.handle, *sub.ptrs(), nthreads, C.byref(out)))
    dt = time.perf_counter() - t0
    exact_bytes = _raw(out)
    model = cpu_model()
    _, share = cpu_share()
    exact = {"value": round(nb / dt / 1e9, 4), "unit": "GB/s", "cores": nthreads, "kind": "port",
             "cpu": model, "cpu_share": share,
             "sample": "first %d files (%.0f MB) of the same corpus; exact CPU path of "
                       "libtrivy_secret.so (tsg_scan_cpu_batch: per-rule bytes.ToLower keyword "
                       "gate + Go-semantics regexp, scanner.go:341-416 restated), %.1f s"
                       % (nf, nb / 1e6, dt)}
    from trivy_amd.secret import GpuContext
    ctx = GpuContext(sc, 0, emulate=True, host_threads=nthreads)
    out = C.c_void_p()
    t0 = time.perf_counter()
    N.check(L.tsg_scan_batch(ctx.handle, *sub.ptrs(), C.byref(out)))
    dt2 = time.perf_counter() - t0
    L.tsg_result_free(out)
    ctx.close()
    opt = {"value": round(nb / dt2 / 1e9, 4), "unit": "GB/s", "cores": nthreads, "kind": "port",
           "cpu": model,
           "sample": "same %.0f MB; the GPU algorithm (K1 automaton, gates, K2 DFAs) emulated "
                     "on the CPU + the same exact resolution (TSG_CTX_EMULATE), %.1f s"
                     % (nb / 1e6, dt2)}
    return exact, opt, sub, exact_bytes


def _raw(out):
    """The bytes of a tsg_result (freed)."""
    from trivy_amd import _native as N
    import ctypes as C
    n = C.c_size_t()
    p = N.lib().tsg_result_data(out, C.byref(n))
    b = C.string_at(p, n.value)
    N.lib().tsg_result_free(out)
    return b


def _summary(out):
    """(files with findings, findings) of a tsg_result."""
    from trivy_amd import _native as N
    import ctypes as C
    ff, nf = C.c_uint64(), C.c_uint64()
    N.check(N.lib().tsg_result_summary(out, None, C.byref(ff), C.byref(nf)))
    return ff.value, nf.value


def kernel_source_sha():
    """sha256 of the device code (HIP sources and the headers they include)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "trivy_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + [os.path.join(csrc, "device.hpp")]):
        h.update(open(f, "rb").read())
    return h.hexdigest()


def _traffic_record(rules, batch_bytes):
    """The FETCH_SIZE record of this rule set when it was measured on the same device code
    and batch size (else None)."""
    path = os.path.join(PMC_DIR, "%s.json" % rules)
    if not os.path.exists(path):
        return None
    m = json.load(open(path))
    if m.get("kernels_sha256") != kernel_source_sha() or int(m.get("batch_bytes", -1)) != int(batch_bytes):
        return None
    return m


def rule_set(name):
    """(scanner, extra plant lines, binary fraction, workload text, rule count)."""
    from trivy_amd import configs
    from trivy_amd import secret as S
    import numpy as np
    if name == "builtin":
        return (S.NewScanner(None), None, 0.0,
                "builtin rules over %.1f GiB synthetic text corpus per GPU (BASELINE configs[1])", 83)
    if name == "user1000":
        doc = configs.user_rules_doc(1000, seed=4)
        sc = S.NewScanner(S.config_from_dict(doc))
        extra = configs.plant_lines(doc, np.random.default_rng(4), 4096)
        return (sc, extra, 0.0,
                "83 builtin + 1,000 user rules (generic clones, keyword-less, unbounded, DFA "
                "blow-up; configs.user_rules_doc) over %.1f GiB synthetic text corpus per GPU "
                "(BASELINE configs[3])", len(sc.Rules))
    doc = configs.allow_exclude_doc()
    sc = S.NewScanner(S.config_from_dict(doc))
    extra = configs.plant_lines(doc, np.random.default_rng(5), 4096)
    extra += ["--- ignore block start ---\nAKIAQWERTYUIOPASDFGH\n--- ignore block stop ---",
              "-----BEGIN IGNORE-----\nglpat-abcdefghij0123456789\n-----END IGNORE-----",
              "aws_access_key_id = AKIAQWERTYUIOPEXAMPLEKEY"]
    return (sc, extra, 0.15,
            "builtin + custom rules with global / per-rule allow rules and exclude blocks over "
            "%.1f GiB per GPU of text files and binary blobs that pass IsBinary (15%% of files; "
            "BASELINE configs[4] shape)", len(sc.Rules))


def fill_slots(ctx, batch, batch_bytes):
    """Pack the corpus into pinned slots of about batch_bytes each (outside timing)."""
    import numpy as np
    slots = []
    f0 = 0
    while f0 < batch.nfiles:
        base = int(batch.offsets[f0])
        f1 = int(np.searchsorted(batch.offsets, base + batch_bytes, side="right")) - 1
        f1 = max(f1, f0 + 1)
        f1 = min(f1, batch.nfiles)
        nb = int(batch.offsets[f1]) - base
        pbase = int(batch.path_offsets[f0])
        npb = int(batch.path_offsets[f1]) - pbase
        sid, data, offs, paths, poffs = ctx.acquire_slot(nb, f1 - f0, npb)
        data[:nb] = batch.data[base:base + nb]
        offs[:f1 - f0 + 1] = batch.offsets[f0:f1 + 1] - np.uint64(base)
        paths[:npb] = batch.paths[pbase:pbase + npb]
        poffs[:f1 - f0 + 1] = batch.path_offsets[f0:f1 + 1] - np.uint64(pbase)
        slots.append((sid, f1 - f0, nb))
        f0 = f1
    return slots


def _visible_gpus():
    """HIP devices this process can see (counting does not initialise the GPU)."""
    try:
        import torch
        return torch.cuda.device_count()
    except ImportError:
        return 0


class DeviceRun:
    """One device's share of the job: its context, its pinned slots (filled before timing),
    and the pipelined submit / collect loop over them."""

    def __init__(self, ctx, slots, info, depth, log):
        self.ctx, self.slots, self.info, self.depth, self.log = ctx, slots, info, depth, log
        self.step_findings = []  # (files with findings, findings) of every step, warmup included

    def run(self, steps, verbose=True):
        """`steps` scans of the share, pipelined across step boundaries (batches of step k+1
        are submitted while step k's last ones resolve); every result is collected."""
        import collections
        import ctypes as C
        from trivy_amd import _native as N
        L = N.lib()
        q = collections.deque()
        per_step = [[0, 0] for _ in range(steps)]

        def collect():
            t, k = q.popleft()
            out = C.c_void_p()
            N.check(L.tsg_batch_collect(self.ctx.handle, t, C.byref(out)))
            ff, nf = _summary(out)
            L.tsg_result_free(out)
            per_step[k][0] += ff
            per_step[k][1] += nf

        for k in range(steps):
            if verbose:
                self.log("step %d/%d" % (k + 1, steps))
            for sid, nf, _ in self.slots:
                t = C.c_uint64()
                N.check(L.tsg_slot_submit(self.ctx.handle, sid, nf, C.byref(t)))
                q.append((t.value, k))
                while len(q) >= self.depth:
                    collect()
        while q:
            collect()
        self.step_findings.extend(tuple(x) for x in per_step)

    def release(self):
        for sid, _, _ in self.slots:
            self.ctx.release_slot(sid)


STAT_SUMS = ("batches", "sum_bytes", "sum_k1_ms", "sum_gate_ms", "sum_k2_ms", "sum_h2d_ms", "sum_d2h_ms",
             "sum_resolve_ms", "sum_prep_ms", "sum_meta_ms", "sum_k1_clock_ms", "sum_chain_clock_ms",
             "sum_post_k1_clock_ms")


def _gbs(nbytes, ms):
    """GB/s, or None without a time (emulated contexts record no kernel times)"""
    return nbytes / (ms / 1e3) / 1e9 if ms else None


def _frac(gbs):
    return round(gbs / HBM_PEAK_GBS, 4) if gbs is not None else None


def _r(x, n=1):
    return round(x, n) if x is not None else None


def _delta(st, st0):
    return {k: st[k] - st0[k] for k in STAT_SUMS}


def _device_ms(d):
    """All of a batch's device work but the batch's own H2D and the wait for the other
    lane: the metadata H2D, prep, K1 (+K1X), gates, K2 and the outputs kernel."""
    return d["sum_meta_ms"] + d["sum_prep_ms"] + d["sum_k1_ms"] + d["sum_gate_ms"] + d["sum_k2_ms"] + d["sum_d2h_ms"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs: under torchrun one rank per GPU (WORLD_SIZE must equal it); "
                         "otherwise this one process drives devices 0..N-1 (tsg_multi)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gb", type=float, default=10.0, help="GiB of corpus per GPU")
    ap.add_argument("--batch-mib", type=int, default=1024, help="bytes per pinned slot / batch")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--depth", type=int, default=4, help="batches in flight per GPU")
    ap.add_argument("--host-threads", type=int, default=0,
                    help="host resolution pool threads (0: library default, 16)")
    ap.add_argument("--cpu-mib", type=int, default=1024, help="CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --gb is the whole job's corpus, split over the GPUs "
                         "(each generates and scans its 1/N share); default: --gb per GPU")
    ap.add_argument("--rules", default="builtin", choices=["builtin", "user1000", "allow-exclude"],
                    help="rule set: builtin (configs[1]), builtin + 1,000 user rules "
                         "(configs[3]), allow rules + exclude blocks over text and binary "
                         "blobs (configs[4])")
    ap.add_argument("--emulate", action="store_true",
                    help="tests only: emulated contexts (the kernels' algorithm on the CPU), no GPU")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="rehearsal only (not a measurement): under torchrun, rank r drives GPU "
                         "r %% visible, so the multi-rank path runs on a box with fewer GPUs; "
                         "the line is marked \"rehearsal\"")
    ap.add_argument("--e2e", choices=["fs", "layer"], default=None,
                    help="end-to-end ingest + scan instead of the configs[1] line: 'fs' = a "
                         "seeded source tree on disk (configs[0] shape, --e2e-mib), 'layer' = a "
                         "seeded layer tar in memory (configs[2] shape); each step walks, gates "
                         "(Required, IsBinary), packs straight into a pinned slot and scans")
    ap.add_argument("--e2e-mib", type=int, default=0, help="e2e input size (default fs 200, layer 2048)")
    ap.add_argument("--e2e-slot-mib", type=int, default=0, help="e2e piece / slot size (0: 256)")
    ap.add_argument("--binary-frac", type=float, default=0.0,
                    help="e2e fs: share of the tree's bytes that are binary blobs (configs[4]: 0.3)")
    ap.add_argument("--binary-text-head", type=float, default=0.5,
                    help="e2e fs: share of the binary blobs that start with 300 bytes of text, so "
                         "IsBinary passes them to Scan (configs[4]: 0.5)")
    ap.add_argument("--piece-mib", type=int, default=0,
                    help="e2e: piece floor of tsg_fs_scan / tsg_layer_scan (the 'piece_mib' test knob; "
                         "0: the library's 16)")
    args = ap.parse_args()
    if args.e2e:
        return main_e2e(args)

    T0 = time.perf_counter()
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1 and args.gpus != ws:  # (before any rendezvous)
        raise SystemExit("bench: --gpus %d under torchrun with WORLD_SIZE=%d: one rank per GPU, "
                         "so they must be equal" % (args.gpus, ws))
    dist, rank, world, local = _dist()
    # devices this process drives: its rank's GPU, or 0..N-1 in one process
    devices = [local] if world > 1 else list(range(args.gpus))
    ngpus = world if world > 1 else args.gpus
    if not args.emulate:
        vis = _visible_gpus()
        if args.rehearse_shared_gpu and world > 1 and vis > 0:
            local = local % vis
            devices = [local]
        if vis < max(devices) + 1:
            raise SystemExit("bench: --gpus %d needs device %d, but this process sees %d GPU(s); "
                             "refusing to run on fewer" % (args.gpus, max(devices), vis))
        if world > 1:  # the barrier's torch.cuda.synchronize() on this rank's GPU, not GPU 0
            import torch
            torch.cuda.set_device(local)
    from trivy_amd import corpus
    from trivy_amd import secret as S
    from trivy_amd import _native as N
    L = N.lib()

    def log(msg):
        print("[bench rank %d %.1fs] %s" % (rank, time.perf_counter() - T0, msg), file=sys.stderr, flush=True)

    nbytes = int(args.gb * (1 << 30) / (ngpus if args.strong else 1))  # per GPU
    t0 = time.perf_counter()
    sc, extra, binary_frac, workload, nrules = rule_set(args.rules)
    compile_s = time.perf_counter() - t0
    batch_bytes = args.batch_mib << 20
    nslots = -(-nbytes // batch_bytes) + 2
    multi = None
    if len(devices) > 1 or args.emulate:
        multi = S.MultiGpu(sc, devices, host_threads=args.host_threads, emulate=args.emulate,
                           max_slots=nslots + 2, chunk_bytes=args.chunk)
        ctxs = [multi.context(i) for i in range(len(devices))]
    else:
        ctxs = [S.GpuContext(sc, devices[0], chunk_bytes=args.chunk, host_threads=args.host_threads,
                             max_slots=nslots + 2)]
    # each GPU's share: a corpus of its own (seeded by its global GPU index), packed into that
    # device's pinned slots before timing; the first GPU's stays for the CPU sample
    runs, gen_s, pack_s, batch0, info0 = [], 0.0, 0.0, None, None
    for i, ctx in enumerate(ctxs):
        g = rank if world > 1 else i
        t0 = time.perf_counter()
        batch, info = corpus.make_corpus(nbytes, seed=args.seed + 1000 * g, plants_per_mib=1.0,
                                         extra_plants=extra, extra_per_mib=2.0 if extra else 0.0,
                                         binary_frac=binary_frac)
        gen_s += time.perf_counter() - t0
        t0 = time.perf_counter()
        slots = fill_slots(ctx, batch, batch_bytes)
        pack_s += time.perf_counter() - t0
        runs.append(DeviceRun(ctx, slots, info, args.depth, log))
        if i == 0:
            info0, batch0 = info, batch
        batch = None
        log("GPU %d: corpus %.2f GiB (%d files), packed" % (devices[i], info["bytes"] / (1 << 30), info["files"]))
    log("generated in %.1fs, rules compiled in %.1fs, packed in %.1fs" % (gen_s, compile_s, pack_s))

    import ctypes as C
    import threading

    def run_all(steps):
        """every device's share, one host thread per device (the native calls release the GIL)"""
        if len(runs) == 1:
            runs[0].run(steps)
            return
        errs = []

        def one(r, verbose):
            try:
                r.run(steps, verbose)
            except BaseException as e:  # noqa: BLE001 (re-raised below)
                errs.append(e)
        th = [threading.Thread(target=one, args=(r, i == 0)) for i, r in enumerate(runs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]

    run_all(args.warmup)
    st0 = [r.ctx.stats() for r in runs]
    _barrier(dist)
    t0 = time.perf_counter()
    run_all(args.steps)
    _barrier(dist)
    dt = time.perf_counter() - t0
    st = [r.ctx.stats() for r in runs]
    dt = _reduce(dist, dt, "MAX")
    local_bytes = float(sum(r.info["bytes"] for r in runs))
    total_bytes = _reduce(dist, local_bytes, "SUM") * args.steps
    ds = [_delta(a, b) for a, b in zip(st, st0)]
    # pooled over this process's devices (per-batch means), and per device for the aggregate
    d = {k: sum(x[k] for x in ds) for k in STAT_SUMS}
    nbat = max(1, d["batches"])
    k1_gbs = _gbs(d["sum_bytes"], d["sum_k1_ms"])
    kern_ms = d["sum_k1_ms"] + d["sum_gate_ms"] + d["sum_k2_ms"]
    dev_ms = _device_ms(d)
    launch_bytes = d["sum_bytes"] / nbat
    # SURVEY §8d aggregate: N_total / max_g(t_g) / (8 TB/s x G), t_g = a GPU's device time
    # over the timed steps (K1 alone, K1 + gates + K2, and all device work)
    agg = {}
    for key, fn in (("k1", lambda x: x["sum_k1_ms"]),
                    ("k1_gates_k2", lambda x: x["sum_k1_ms"] + x["sum_gate_ms"] + x["sum_k2_ms"]),
                    ("device", _device_ms)):
        tmax = _reduce(dist, max(fn(x) for x in ds), "MAX") / 1e3
        agg[key + "_frac"] = round(total_bytes / tmax / (HBM_PEAK_GBS * 1e9 * ngpus), 4) if tmax else None
    last = st[0]
    k2_read = last["k2_bytes"]  # last batch of the first device: chunk bytes K2 read
    pmc = _traffic_record(args.rules, int(launch_bytes))
    k1_name = ("K1F keyword/anchor filter + exact verification and run counters (k1f_kernel)"
               if last["k1_filter"] else "K1 keyword automaton (k1_kernel)")
    if last["k1x_records"]:  # a large rule set: K1X ran after K1, inside the same K1 events
        k1_name += " + K1X hashed prefilter and verify (k1x_kernel, k1x_verify_kernel)"
    if pmc and pmc.get("k1_kernel", "k1_kernel") != ("k1f_kernel" if last["k1_filter"] else "k1_kernel"):
        pmc = None  # a pass of the other K1
    ngpus_s = "x%d" % ngpus
    line = {
        "metric": "secret-scan GB/s (builtin rules) at 1/2/4/8 MI355X; % of HBM peak",
        "value": round(total_bytes / dt / 1e9, 3),
        "unit": "GB/s",
        "n_gpus": ngpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded corpus per GPU, trivy_amd/corpus.py) in pinned host memory; every "
                "step moves every byte host->HBM (H2D inside the timed region)",
        "config": {"workload": workload % (nbytes / (1 << 30)) + (
                       "; strong scaling: a %.1f GiB job split over %d GPUs" % (args.gb, ngpus)
                       if args.strong else ""),
                   "files_per_gpu": info0["files"], "bytes_per_gpu": info0["bytes"],
                   "job_bytes": int(total_bytes / args.steps),
                   "batches_per_step": sum(len(r.slots) for r in runs), "batch_bytes": batch_bytes,
                   "rules": nrules,
                   "parallelism": ("file-sharded %s, one process per GPU (torchrun), no collective" % ngpus_s
                                   if world > 1 else
                                   "file-sharded %s, one process driving %d device(s) (tsg_multi), no "
                                   "collective" % (ngpus_s, len(devices))) + (
                                       ", EMULATED contexts (no GPU)" if args.emulate else ""),
                   "devices": devices if world == 1 else None},
        "roofline": {"bound": "hbm", "kernel": k1_name,
                     "achieved": _r(k1_gbs), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": _frac(k1_gbs),
                     "traffic": pmc["k1_bytes_per_launch"] if pmc else None,
                     "algorithmic_bytes_per_launch": int(launch_bytes),
                     "traffic_source": pmc["csv"] if pmc else
                     "none: no FETCH_SIZE pass of this device code, rule set and batch size "
                     "in profiles/pmc/",
                     "traffic_calibration": (
                         "FETCH_SIZE KiB x 1024 / %s (%s; profiles/pmc/fetch_calib.json)" % (
                             pmc.get("fetch_factor", 0.922),
                             "16 contiguous bytes per lane" if pmc.get("k1_kernel") == "k1f_kernel"
                             else "quad-transposed 64-B loads")) if pmc else None,
                     "k1_listed_words_last_batch": last["k1f_listed"] if last["k1_filter"] else None,
                     "k1_verified_arrivals_last_batch": last["k1f_arrivals"] if last["k1_filter"] else None,
                     "k1_gates_k2_frac": _frac(_gbs(d["sum_bytes"], kern_ms)),
                     # the same spans by the device wall clock stamped inside the kernels (first
                     # block start to last block end, tsg_stats.*_clock_ms): frac_clock is K1's,
                     # chain_frac_clock K1's start to K2's end, every kernel and gap between
                     "frac_events": _frac(k1_gbs),
                     "frac_clock": _frac(_gbs(d["sum_bytes"], d["sum_k1_clock_ms"])),
                     "chain_frac_clock": _frac(_gbs(d["sum_bytes"], d["sum_chain_clock_ms"])),
                     "k1_clock_ms_per_batch": round(d["sum_k1_clock_ms"] / nbat, 4),
                     "chain_clock_ms_per_batch": round(d["sum_chain_clock_ms"] / nbat, 4),
                     "post_k1_clock_ms_per_batch": round(d["sum_post_k1_clock_ms"] / nbat, 4),
                     "device_frac": _frac(_gbs(d["sum_bytes"], dev_ms)),
                     "aggregate": dict(agg, gpus=ngpus,
                                       definition="job bytes / max over GPUs of that GPU's device "
                                                  "ms (HIP events) / (8 TB/s x GPUs)")},
        "kernels": {"k1_GBps": _r(k1_gbs),
                    "k2_GBps_on_item_bytes": round(k2_read / (last["k2_ms"] / 1e3) / 1e9, 1)
                    if last["k2_ms"] else None,
                    "k1_gates_k2_GBps": _r(_gbs(d["sum_bytes"], kern_ms)),
                    "device_GBps": _r(_gbs(d["sum_bytes"], dev_ms)),
                    "device_ms_per_batch": round(dev_ms / nbat, 4),
                    "meta_h2d_ms_per_batch": round(d["sum_meta_ms"] / nbat, 4),
                    "prep_ms_per_batch": round(d["sum_prep_ms"] / nbat, 4),
                    "k1_ms_per_batch": round(d["sum_k1_ms"] / nbat, 4),
                    "gates_ms_per_batch": round(d["sum_gate_ms"] / nbat, 4),
                    "k2_ms_per_batch": round(d["sum_k2_ms"] / nbat, 4),
                    "outputs_ms_per_batch": round(d["sum_d2h_ms"] / nbat, 4),
                    "per_device": [{"device": dv, "batches": x["batches"],
                                    "k1_ms": round(x["sum_k1_ms"], 3),
                                    "k1_gates_k2_ms": round(x["sum_k1_ms"] + x["sum_gate_ms"] + x["sum_k2_ms"], 3),
                                    "device_ms": round(_device_ms(x), 3)}
                                   for dv, x in zip(devices, ds)],
                    "k2_item_bytes_last_batch": k2_read, "k2_entries_last_batch": last["k2_launches"],
                    "candidates_last_batch": last["candidates"],
                    "groups_skipped_last_batch": last["groups_skipped"],
                    "k2_diag_last_batch": {k: last[k] for k in ("k2_tail_bytes", "k2_tail_max",
                                                                 "k2_long_tails", "k2_replays")}},
        "pipeline": {"h2d_GBps": _r(_gbs(d["sum_bytes"], d["sum_h2d_ms"]), 2),
                     "h2d_ms_per_batch": round(d["sum_h2d_ms"] / nbat, 3),
                     "resolve_ms_per_batch": round(d["sum_resolve_ms"] / nbat, 3),
                     "depth": args.depth, "lanes": 2,
                     "gen_s": round(gen_s, 2), "pack_into_pinned_s": round(pack_s, 2),
                     "rule_compile_s": round(compile_s, 2)},
    }
    if args.rehearse_shared_gpu:
        # ranks share GPUs: the line cannot claim more GPUs than it used, nor a multi-GPU rate
        distinct = min(world, _visible_gpus()) if not args.emulate else 1
        line["rehearsal"] = {"note": "ranks share GPUs (--rehearse-shared-gpu): not a measurement",
                             "ranks": world, "distinct_gpus": distinct}
        line["n_gpus"] = distinct
        line["value"] = None
        line["vs_baseline"] = None
        line["roofline"]["aggregate"] = None
    log("timed %d steps: %.3f s" % (args.steps, dt))
    # every step of every device must have produced the same findings as its warmup steps
    # (the timed loop reads every result)
    for dv, r in zip(devices, runs):
        if len(set(r.step_findings)) != 1:
            raise SystemExit("bench: findings differ between steps on device %d: %s" % (dv, r.step_findings))
    line["checks"] = {"findings_per_step": sum(r.step_findings[0][1] for r in runs),
                      "files_with_findings_per_step": sum(r.step_findings[0][0] for r in runs),
                      "steps_checked": len(runs[0].step_findings)}
    if rank == 0 and not args.no_cpu_baseline:
        nt = args.host_threads or cpu_share()[0]
        exact, opt, sub, exact_bytes = cpu_baselines(sc, batch0, args.cpu_mib << 20, nt)
        # (a one-GPU figure: reported at N=1; at N>1 the sample only checks the device)
        line["cpu_baseline"], line["cpu_optimised"] = (exact, opt) if ngpus == 1 else (None, None)
        out = C.c_void_p()
        N.check(L.tsg_scan_batch(ctxs[0].handle, *sub.ptrs(), C.byref(out)))
        if _raw(out) != exact_bytes:
            raise SystemExit("bench: the device result of the cpu_baseline sample differs from "
                             "the exact CPU path")
        line["checks"]["sample_device_eq_exact_cpu"] = True
        line["checks"]["sample_files"] = sub.nfiles
    for r in runs:
        r.release()
    for c in ctxs:
        c.close()
    if multi is not None:
        multi.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main_e2e(args):
    """ingest -> findings on one GPU, every stage inside the timed step.
    One step = one tsg_fs_scan / tsg_layer_scan call: walk, Required, IsBinary, the kept
    files written straight into pinned slots in pieces of the context's slot size, each piece
    uploaded, scanned and resolved while the next is written; the step ends with the
    serialized per-file results of every kept file in the library's result buffer.  The
    first step's result bytes must equal the exact CPU path's over the pageable pack of the
    same input, and every step must find the same.  An unpipelined step (the pack into one
    slot, then its scan) is timed once beside it for the stage breakdown."""
    import ctypes as C
    import shutil
    import tempfile
    from trivy_amd import _native as N
    from trivy_amd import analyzer as A
    from trivy_amd import configs
    from trivy_amd import secret as S
    from trivy_amd import walker as W
    L = N.lib()
    if args.piece_mib:
        N.knob("piece_mib", args.piece_mib)
    tmp = tempfile.mkdtemp(prefix="tsg_e2e_")
    an = A.SecretAnalyzer()
    extra = None
    if args.rules == "builtin":
        an.Init("")
    else:  # the rule set as a trivy-secret.yaml outside the scanned input (secret.go:62-76)
        import numpy as np
        import yaml
        doc = configs.user_rules_doc(1000, seed=4) if args.rules == "user1000" else configs.allow_exclude_doc()
        cfg_path = os.path.join(tmp, "trivy-secret.yaml")
        with open(cfg_path, "w") as f:
            yaml.safe_dump(doc, f)
        an.Init(cfg_path)
        extra = rule_set(args.rules)[1]
    sc = an.scanner
    mib = args.e2e_mib or (200 if args.e2e == "fs" else 2048)
    cfg = an.configPath.encode()
    none = (C.c_char_p * 1)()
    t0 = time.perf_counter()
    tree_info = None
    if args.e2e == "fs":
        root = os.path.join(tmp, "tree")
        tree_info = configs.source_tree(root, mib << 20, seed=args.seed, binary_frac=args.binary_frac,
                                        binary_text_head=args.binary_text_head, extra_plants=extra,
                                        extra_per_mib=2.0 if extra else 0.0)
        in_bytes = sum(os.path.getsize(os.path.join(d, f)) for d, _, fs in os.walk(root) for f in fs)

        def one_call(ctx, out):
            h = C.c_void_p()
            N.check(L.tsg_fs_scan(ctx.handle, root.encode(), none, 0, none, 0, cfg, C.byref(h), C.byref(out)))
            L.tsg_layer_free(h)
        unpiped = lambda ctx: W.SlotIngest.fs(ctx, root, config_path=an.configPath)  # noqa: E731
        ref = W.NativeFS(sc, root, config_path=an.configPath)
        what = "seeded source tree on local disk (page cache warm), %d MiB, configs[0] shape" % mib
        if args.binary_frac:
            what += ("; %.0f%% of the bytes binary blobs (%d files, %d with a text head that IsBinary "
                     "passes, the rest dropped), configs[4] mix" % (
                         100 * args.binary_frac, tree_info["binary_files"], tree_info["binary_text_head_files"]))
    else:
        tar = configs.layer_tar(mib << 20, seed=args.seed)
        in_bytes = len(tar)
        import numpy as np
        tarr = np.frombuffer(tar, dtype=np.uint8)

        def one_call(ctx, out):
            h = C.c_void_p()
            N.check(L.tsg_layer_scan(ctx.handle, C.c_void_p(tarr.ctypes.data), len(tar), none, 0, none, 0, cfg,
                                     C.byref(h), C.byref(out)))
            L.tsg_layer_free(h)
        unpiped = lambda ctx: W.SlotIngest.layer(ctx, tar, config_path=an.configPath)  # noqa: E731
        ref = W.NativeLayer(sc, tar, config_path=an.configPath)
        what = "seeded uncompressed layer tar in host memory, %d MiB, configs[2] shape" % mib
    gen_s = time.perf_counter() - t0
    ctx = S.GpuContext(sc, 0, host_threads=args.host_threads, slot_mib=args.e2e_slot_mib, emulate=args.emulate)
    scanned = int(ref.batch.offsets[-1])

    def step(check=False):
        out = C.c_void_p()
        one_call(ctx, out)
        summ = _summary(out)
        return summ, (_raw(out) if check else L.tsg_result_free(out))

    for _ in range(max(1, args.warmup)):
        summ0, raw0 = step(check=True)
    out = C.c_void_p()
    t0 = time.perf_counter()
    N.check(L.tsg_scan_cpu_batch(sc.handle, *ref.batch.ptrs(), args.host_threads or cpu_share()[0], C.byref(out)))
    cpu_s = time.perf_counter() - t0
    if raw0 != _raw(out):
        raise SystemExit("bench --e2e: device results differ from the exact CPU path")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        summ, _ = step()
        if summ != summ0:
            raise SystemExit("bench --e2e: findings differ between steps")
    dt = time.perf_counter() - t0
    # stage breakdown, unpipelined: the whole input packed into one slot, then scanned
    a = time.perf_counter()
    g = unpiped(ctx)
    b = time.perf_counter()
    tk, out = C.c_uint64(), C.c_void_p()
    N.check(L.tsg_slot_submit(ctx.handle, g._slot, g.batch.nfiles, C.byref(tk)))
    N.check(L.tsg_batch_collect(ctx.handle, tk.value, C.byref(out)))
    c = time.perf_counter()
    if _summary(out) != summ0:
        raise SystemExit("bench --e2e: the unpipelined scan finds something else")
    L.tsg_result_free(out)
    g.release()
    ctx.close()
    shutil.rmtree(tmp, ignore_errors=True)
    line = {"metric": "end-to-end secret scan (ingest + scan) GB/s of input, 1 MI355X",
            "value": round(in_bytes * args.steps / dt / 1e9, 3), "unit": "GB/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: " + what,
            "config": {"workload": "e2e-" + args.e2e + ("" if args.rules == "builtin" else "-" + args.rules),
                       "input_bytes": in_bytes, "scanned_bytes": scanned,
                       "files_scanned": ref.batch.nfiles, "findings": summ0[1], "rules": len(sc.Rules),
                       "rule_set": args.rules, "binary_frac": args.binary_frac,
                       "piece_mib": args.e2e_slot_mib or 256,
                       "api": "tsg_fs_scan" if args.e2e == "fs" else "tsg_layer_scan"},
            "unpipelined": {"ingest_ms": round((b - a) * 1e3, 2),
                            "ingest_GBps_of_input": round(in_bytes / (b - a) / 1e9, 3),
                            "scan_ms": round((c - b) * 1e3, 2),
                            "scan_GBps_of_scanned": round(scanned / (c - b) / 1e9, 3)},
            "cpu_baseline": {"value": round(scanned / cpu_s / 1e9, 4), "unit": "GB/s of scanned bytes",
                             "cores": args.host_threads or cpu_share()[0], "kind": "port",
                             "cpu_share": cpu_share()[1],
                             "sample": "the whole packed input; exact CPU path (tsg_scan_cpu_batch)"},
            "gen_s": round(gen_s, 2),
            "checks": {"step1_eq_exact_cpu": True, "findings_per_step": summ0[1],
                       "files_with_findings_per_step": summ0[0]}}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
