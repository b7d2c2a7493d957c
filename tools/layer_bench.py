#!/usr/bin/env python3
"""configs[2]-shaped measurement (not the bench.py headline): one seeded image-layer tar
(trivy_amd.configs.layer_tar) through the native ingest (tsg_layer_pack: tar walk +
Required + IsBinary + packing) and a GPU scan of the packed batch.

    python tools/layer_bench.py [GiB] [scans]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from trivy_amd import analyzer as A  # noqa: E402
from trivy_amd import configs  # noqa: E402
from trivy_amd import secret as S  # noqa: E402
from trivy_amd import walker as W  # noqa: E402


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    scans = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    t0 = time.time()
    tar = configs.layer_tar(int(gib * (1 << 30)), seed=3)
    gen_s = time.time() - t0
    an = A.SecretAnalyzer(S.NewScanner(None), "")
    packs = []
    for _ in range(3):
        t = time.perf_counter()
        lay = W.NativeLayer(an.scanner, tar)
        packs.append(time.perf_counter() - t)
    b = lay.batch
    scanned = int(b.offsets[-1])
    ctx = S.GpuContext(an.scanner, 0)
    t = time.perf_counter()
    ctx.upload(b)
    up_s = time.perf_counter() - t
    an.scanner.ScanBatch(b, ctx=ctx)  # warm-up (adaptation pass)
    times = []
    for _ in range(scans):
        t = time.perf_counter()
        res = an.scanner.ScanBatch(b, ctx=ctx)
        times.append(time.perf_counter() - t)
    nfind = sum(len(r["Findings"] or []) for r in res)
    # configs[2] over W GPUs: (a) every rank indexes the whole chain and packs only its byte
    # run (tsg_layer_pack_shard); the slowest rank's pack time, measured here rank by rank
    shard = {}
    for world in (2, 4, 8):
        worst = 0.0
        for rank in range(world):
            t = time.perf_counter()
            W.NativeLayer(an.scanner, tar, rank=rank, world=world)
            worst = max(worst, time.perf_counter() - t)
        # distributed index (tsg_layer_range_*): each rank walks only its byte range; the
        # exchange is simulated in-process (layer_chain_step); per-rank time = its walk +
        # sync + dirs + pack, measured rank by rank
        rngs, walk_t = [], []
        for rank in range(world):
            t = time.perf_counter()
            rngs.append(W.LayerRange(tar, rank, world))
            walk_t.append(time.perf_counter() - t)
        infos, confirmed = [g.info for g in rngs], {}
        while True:
            st = W.layer_chain_step(infos, confirmed)
            if st[0] == "done":
                break
            confirmed[st[1]] = rngs[st[1]].sync(st[2])
        worst_r, prior, resync = 0.0, [], len(confirmed)
        for rank, g in enumerate(rngs):
            t = time.perf_counter()
            g.sync(st[1][rank])
            d = g.dirs()
            lay_r = g.pack(an.scanner, (), (), prior, "")
            worst_r = max(worst_r, walk_t[rank] + time.perf_counter() - t)
            prior = prior + d
            del lay_r
        shard[str(world)] = {"slowest_rank_pack_s": round(worst, 4),
                             "per_rank_ingest_GBps_of_tar": round(len(tar) / worst / 1e9, 2),
                             "range_index_slowest_rank_s": round(worst_r, 4),
                             "range_index_per_rank_GBps_of_tar": round(len(tar) / worst_r / 1e9, 2),
                             "range_index_resyncs": resync}
    pack_s = min(packs)
    scan_s = min(times)
    print(json.dumps({
        "workload": "seeded layer tar %.2f GiB (configs[2] shape, 1 GPU)" % gib,
        "tar_bytes": len(tar), "walked": lay.walked, "scanned_files": b.nfiles,
        "scanned_bytes": scanned, "findings": nfind,
        "ingest_GBps_of_tar": len(tar) / pack_s / 1e9, "ingest_s": pack_s,
        "scan_s_incl_h2d_and_resolve": scan_s, "scan_GBps": scanned / scan_s / 1e9,
        "upload_s": up_s, "gen_s": gen_s,
        "layer_e2e_GBps_of_tar": len(tar) / (pack_s + scan_s) / 1e9,
        "sharded_pack": shard}))


if __name__ == "__main__":
    main()
