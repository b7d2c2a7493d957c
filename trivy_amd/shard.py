"""File sharding across GPUs of one node.

Files are independent units of `Scanner.Scan` (pkg/fanal/secret/scanner.go:341), so a
node-wide scan needs no collective on the data path.  Each rank (one process per GPU)
scans an LPT bin-packed share of the files by bytes; the sparse results are gathered on
rank 0 and sorted by path as `AnalysisResult.Sort` does (pkg/fanal/analyzer/analyzer.go:
212-223).  The gather is host-side (torch.distributed object collectives over gloo); no
RCCL traffic.
"""
import heapq

from . import secret as S


def lpt_shards(sizes, world):
    """Longest-processing-time bin packing: file indices per rank, each list ascending."""
    heap = [(0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
    return [sorted(x) for x in out]


def scan_sharded(scanner, args, rank, world, dist=None, device=None, emulate_chunk=0):
    """Scan `args` (the same list on every rank) sharded over `world` ranks.

    Rank r scans its LPT share (on `device` when given, else the emulated kernel path
    when emulate_chunk > 0, else the exact CPU path); rank 0 returns the results for
    every file in input order, the other ranks return None."""
    shards = lpt_shards([len(a.Content) for a in args], world)
    mine = shards[rank]
    local = scanner.ScanBatch([args[i] for i in mine], device=device,
                              emulate_chunk=emulate_chunk) if mine else []
    if world == 1 or dist is None:
        return local
    payload = list(zip(mine, local))
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(payload, gathered, dst=0)
    if rank != 0:
        return None
    res = [None] * len(args)
    for part in gathered:
        for i, r in part:
            res[i] = r
    return res


def scan_layer_sharded(analyzer, tar, rank, world, dist=None, device=None, emulate_chunk=0,
                       skip_files=(), skip_dirs=(), index="range"):
    """BASELINE configs[2]: one image layer's files sharded over `world` ranks.

    index="range" (default): the header index itself is split; each rank walks its own byte
    range of the tar and the ranks fix the true chain and the walker's skip dirs with two
    tiny all-gathers (walker.layer_chain, tsg_layer_range_*), then each packs and scans the
    files of its range.  index="whole": every rank indexes the whole chain and packs its
    contiguous byte run of the walked files (tsg_layer_pack_shard).  The findings are
    gathered on rank 0; rank 0 returns (sorted AnalysisResult.Secrets, opq_dirs, wh_files),
    the others None."""
    from .walker import NativeLayer, LayerRange, layer_chain

    def scan(lay):
        b = lay.batch
        if b.nfiles == 0:
            return []
        if device is not None or emulate_chunk:
            return analyzer.scanner.ScanBatch(b, device=device, emulate_chunk=emulate_chunk)
        return analyzer.scanner.ScanBatch(b, nthreads=16)

    if index == "range" and world > 1 and dist is not None:
        def allgather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out

        def guarded(fn):
            """fn() on this rank, then one all-gather of (ok, value) / (err, message): every
            rank raises if any rank failed, so no rank is left waiting in a collective."""
            try:
                mine = ("ok", fn())
            except Exception as e:  # noqa: BLE001 - forwarded to every rank
                mine = ("err", "rank %d: %s" % (rank, e))
            out = allgather(mine)
            bad = [m for k, m in out if k == "err"]
            if bad:
                raise RuntimeError("; ".join(bad))
            return [v for _, v in out]

        holder = {}

        def make_range():
            holder["rng"] = LayerRange(tar, rank, world)
            return None
        guarded(make_range)
        rng = holder["rng"]
        # every rank's range info, gathered in a guarded step of its own: inside layer_chain
        # every collective is then entered by all ranks (its only failures are raised on
        # every rank, after the same all-gathers)
        infos = guarded(lambda: rng.info)

        def chain():
            holder["pos"] = layer_chain(rng, rank, world, allgather, infos=infos)
            return None
        guarded(chain)
        dirs = guarded(lambda: rng.dirs(skip_dirs))
        prior = [d for r in range(rank) for d in dirs[r]]

        def pack_scan():
            holder["lay"] = rng.pack(analyzer.scanner, skip_files, skip_dirs, prior,
                                     analyzer.configPath)
            holder["local"] = scan(holder["lay"])
        guarded(pack_scan)
        lay, local = holder["lay"], holder["local"]
    else:
        lay = NativeLayer(analyzer.scanner, tar, skip_files, skip_dirs, analyzer.configPath,
                          rank=rank, world=world)
        local = scan(lay)
    mine = [r for r in local if r and r["Findings"]]
    if world == 1 or dist is None:
        return findings_sorted(mine), lay.opq, lay.wh
    per_rank = index == "range"  # opq / wh of the range only: concatenated in rank order
    gathered = [None] * world if rank == 0 else None
    dist.gather_object((mine, lay.opq, lay.wh), gathered, dst=0)
    if rank != 0:
        return None
    secrets = findings_sorted([r for part in gathered for r in part[0]])
    if per_rank:
        return (secrets, [d for part in gathered for d in part[1]],
                [w for part in gathered for w in part[2]])
    return secrets, lay.opq, lay.wh


def scan_fs_sharded(analyzer, root, rank, world, dist=None, device=None, emulate_chunk=0,
                    skip_files=(), skip_dirs=()):
    """BASELINE configs[0] over `world` ranks (one process per GPU): every rank lists the
    tree and reads only its contiguous byte run of the listed files (tsg_fs_pack_shard:
    no rank holds another's file contents), scans it, and rank 0 gathers the files with
    findings (sparse) and returns them sorted as AnalysisResult.Sort does; the other ranks
    return None.  A failure on one rank raises on every rank (one status all-gather before
    the gather), so no rank is left waiting in a collective."""
    from .walker import NativeFS

    def pack_scan():
        fs = NativeFS(analyzer.scanner, root, skip_files, skip_dirs, analyzer.configPath,
                      rank=rank, world=world)
        b = fs.batch
        if b.nfiles == 0:
            return []
        if device is not None or emulate_chunk:
            local = analyzer.scanner.ScanBatch(b, device=device, emulate_chunk=emulate_chunk)
        else:
            local = analyzer.scanner.ScanBatch(b, nthreads=16)
        return [r for r in local if r and r["Findings"]]

    if world == 1 or dist is None:
        return findings_sorted(pack_scan())
    mine = None
    try:
        mine = pack_scan()
        status = ("ok", "")
    except Exception as e:  # noqa: BLE001 - forwarded to every rank
        status = ("err", "rank %d: %s" % (rank, e))
    sts = [None] * world
    dist.all_gather_object(sts, status)
    bad = [m for k, m in sts if k == "err"]
    if bad:
        raise RuntimeError("; ".join(bad))
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0)
    if rank != 0:
        return None
    return findings_sorted([r for part in gathered for r in part])


def findings_sorted(results):
    """The secrets of AnalysisResult after Sort: files with findings, by path."""
    from .analyzer import sort_secrets
    return sort_secrets([r for r in results if r and r["Findings"]])


__all__ = ["lpt_shards", "scan_sharded", "scan_layer_sharded", "scan_fs_sharded", "findings_sorted", "S"]
