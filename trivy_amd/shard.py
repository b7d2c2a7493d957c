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
                       skip_files=(), skip_dirs=()):
    """BASELINE configs[2]: one image layer's files sharded over `world` ranks.

    Each rank indexes the layer's header chain and packs only its own contiguous byte run
    of the walked files (tsg_layer_pack_shard: `Required`, `IsBinary` and the copy for that
    run only), scans it, and the findings are gathered on rank 0; rank 0 returns (sorted
    AnalysisResult.Secrets, opq_dirs, wh_files), the others None."""
    from .walker import NativeLayer
    lay = NativeLayer(analyzer.scanner, tar, skip_files, skip_dirs, analyzer.configPath,
                      rank=rank, world=world)
    b = lay.batch
    if b.nfiles == 0:
        local = []
    elif device is not None or emulate_chunk:
        local = analyzer.scanner.ScanBatch(b, device=device, emulate_chunk=emulate_chunk)
    else:
        local = analyzer.scanner.ScanBatch(b, nthreads=16)
    mine = [r for r in local if r and r["Findings"]]
    if world == 1 or dist is None:
        return findings_sorted(mine), lay.opq, lay.wh
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0)
    if rank != 0:
        return None
    return findings_sorted([r for part in gathered for r in part]), lay.opq, lay.wh


def findings_sorted(results):
    """The secrets of AnalysisResult after Sort: files with findings, by path."""
    from .analyzer import sort_secrets
    return sort_secrets([r for r in results if r and r["Findings"]])


__all__ = ["lpt_shards", "scan_sharded", "scan_layer_sharded", "findings_sorted", "S"]
