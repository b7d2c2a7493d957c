#!/usr/bin/env python3
"""Secret-scan throughput on MI355X (BASELINE.json metric, configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--gb G]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (per rank, weak scaling): builtin rules over a seeded synthetic corpus of
--gb GiB (default 10: BASELINE configs[1]) of mixed code/config text files with planted
secrets.  The batch is uploaded to HBM once (outside the timed region); one step =
one scan of the resident batch: K1 keyword automaton, gates, K2 rule-group DFAs,
candidate download (tsg_batch_submit), then exact host resolution of every finding (Go
semantics) and serialization of all per-file results (tsg_batch_collect).  Steps are
pipelined two deep: the device part of step i+1 runs while the host resolves step i.
The timed region ends when every step's results have been collected.
value = content bytes of all ranks x steps / max-over-ranks wall time.

Rank 0 prints ONE JSON line with, in addition to the contract fields:
  roofline      the dominant kernel's algorithmic bytes / its mean HIP-event duration
                (events recorded on the context's stream around each launch) vs 8 TB/s
  cpu_baseline  the oracle (Python restatement of the reference's algorithm) timed on a
                bounded sample of the same corpus on this host, 1 core
  cpu_native    the product library's exact CPU path (C++ restatement of the same
                algorithm: per-rule keyword gate, Go-semantics Pike VM over whole files),
                16 threads, on a bounded sample -- the closer stand-in for Go's speed
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# FETCH_SIZE of the same command (rocprofv3 --pmc FETCH_SIZE), committed under profiles/
PMC_FETCH_CSV = os.path.join(ROOT, "profiles", "r01", "bench_10gib_pmc_fetch_v10.csv")


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return None, 0, 1, 0
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo")
    return dist, dist.get_rank(), ws, int(os.environ.get("LOCAL_RANK", "0"))


def _barrier(dist):
    """Barrier + device sync (the scans run on the library's own HIP stream and each
    submit waits for it; torch's synchronize covers anything else on the device)."""
    if dist is not None:
        dist.barrier()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except ImportError:
        pass


def _max(dist, v):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum(dist, v):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(batch, budget_s=12.0):
    """Oracle (reference algorithm restated in Python) on a bounded prefix of the corpus."""
    from oracle import secret as O
    osc = O.NewScanner(None)
    done = 0
    nfiles = 0
    t0 = time.perf_counter()
    for i in range(batch.nfiles):
        c = bytes(batch.data[int(batch.offsets[i]):int(batch.offsets[i + 1])])
        osc.Scan(batch.path(i), c)
        done += len(c)
        nfiles += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt / 1e9, "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "first %d files (%.2f MB) of the same corpus, oracle/secret.py "
                      "(Go regexp restated over Python `regex`), %.1f s" % (nfiles, done / 1e6, dt)}


def _traffic(dom, gb):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass (same
    10 GiB workload; null for other sizes or when the file is absent)."""
    if abs(gb - 10.0) > 1e-9 or not os.path.exists(PMC_FETCH_CSV):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import traffic
    t = traffic(PMC_FETCH_CSV, "k1_kernel" if dom.startswith("K1") else "k2_")
    return None if t is None else int(t)


def cpu_native(sc, batch, max_bytes=256 << 20, nthreads=16):
    """Exact CPU batch path of libtrivy_secret.so on the first files of the corpus."""
    from trivy_amd import _native as N
    import ctypes as C
    nf = 0
    while nf < batch.nfiles and int(batch.offsets[nf + 1]) <= max_bytes:
        nf += 1
    nf = max(nf, 1)
    from trivy_amd.secret import Batch
    sub = Batch(batch.data[:int(batch.offsets[nf])], batch.offsets[:nf + 1],
                batch.paths[:int(batch.path_offsets[nf])], batch.path_offsets[:nf + 1])
    out = C.c_void_p()
    t0 = time.perf_counter()
    N.check(N.lib().tsg_scan_cpu_batch(sc.handle, *sub.ptrs(), nthreads, C.byref(out)))
    dt = time.perf_counter() - t0
    N.lib().tsg_result_free(out)
    nb = int(batch.offsets[nf])
    return {"value": nb / dt / 1e9, "unit": "GB/s", "cores": nthreads, "kind": "port",
            "sample": "first %d files (%.1f MB) of the same corpus, exact CPU path of "
                      "libtrivy_secret.so (tsg_scan_cpu_batch), %.1f s" % (nf, nb / 1e6, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gb", type=float, default=10.0, help="GiB of corpus per rank")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--depth", type=int, default=4, help="pipelined scans in flight")
    ap.add_argument("--host-threads", type=int, default=0,
                    help="host resolution pool threads (0: library default, 16)")
    args = ap.parse_args()

    dist, rank, world, local = _dist()
    from trivy_amd import corpus
    from trivy_amd import secret as S

    nbytes = int(args.gb * (1 << 30))
    t0 = time.perf_counter()
    batch, info = corpus.make_corpus(nbytes, seed=args.seed + 1000 * rank, plants_per_mib=1.0)
    gen_s = time.perf_counter() - t0
    sc = S.NewScanner(None)
    dev = local if world > 1 else 0
    ctx = S.GpuContext(sc, dev, chunk_bytes=args.chunk, host_threads=args.host_threads)
    t0 = time.perf_counter()
    ctx.upload(batch)
    upload_s = time.perf_counter() - t0
    from trivy_amd import _native as N
    L = N.lib()

    acc = {"k1": 0.0, "k2": 0.0, "gate": 0.0, "res": 0.0, "submit": 0.0, "wait": 0.0}

    def collect():
        t = time.perf_counter()
        L.tsg_result_free(ctx.collect_raw())
        acc["wait"] += (time.perf_counter() - t) * 1e3
        acc["res"] += ctx.stats()["resolve_ms"]

    def run(k):
        for _ in range(k):
            t = time.perf_counter()
            ctx.submit()
            acc["submit"] += (time.perf_counter() - t) * 1e3
            st = ctx.stats()
            acc["k1"] += st["k1_ms"]
            acc["k2"] += st["k2_ms"]
            acc["gate"] += st["gate_ms"]
            while ctx.pending() >= args.depth:
                collect()
        while ctx.pending():
            collect()

    run(args.warmup)
    for k in acc:
        acc[k] = 0.0
    _barrier(dist)
    t0 = time.perf_counter()
    run(args.steps)
    _barrier(dist)
    dt = time.perf_counter() - t0
    dt = _max(dist, dt)
    k1, k2, res = acc["k1"], acc["k2"], acc["res"]
    total_bytes = _sum(dist, float(info["bytes"])) * args.steps
    st = ctx.stats()
    k1_ms, k2_ms = k1 / args.steps, k2 / args.steps
    dom = "K1 keyword automaton" if k1_ms >= k2_ms else "K2 rule-group DFAs (all launches)"
    dom_ms = max(k1_ms, k2_ms)
    achieved = info["bytes"] / (dom_ms / 1e3) / 1e9
    line = {
        "metric": "secret-scan GB/s (builtin rules) at 1/2/4/8 MI355X; % of HBM peak",
        "value": round(total_bytes / dt / 1e9, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded corpus, trivy_amd/corpus.py; resident in HBM)",
        "config": {"workload": "builtin rules over %.1f GiB synthetic text corpus per GPU "
                               "(BASELINE configs[1])" % args.gb,
                   "files_per_gpu": info["files"], "bytes_per_gpu": info["bytes"],
                   "rules": 83, "parallelism": "file-sharded x%d, no collective" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": _traffic(dom, args.gb),
                     "algorithmic_bytes": info["bytes"],
                     "traffic_source": os.path.relpath(PMC_FETCH_CSV, ROOT)},
        "breakdown_ms": {"k1": round(k1_ms, 3), "gate": round(acc["gate"] / args.steps, 3),
                         "k2": round(k2_ms, 3),
                         "resolve": round(res / args.steps, 3), "aux": round(st["aux_ms"], 3),
                         "submit_wall": round(acc["submit"] / args.steps, 3),
                         "collect_wait": round(acc["wait"] / args.steps, 3),
                         "k2_launches": st["k2_launches"], "candidates": st["candidates"],
                         "upload_s": round(upload_s, 3), "gen_s": round(gen_s, 2),
                         "pcie_inclusive_GBps": round(info["bytes"] / (upload_s + dt / args.steps) / 1e9, 3)},
    }
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(batch)
        line["cpu_native"] = cpu_native(sc, batch)
    ctx.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
