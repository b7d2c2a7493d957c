#!/usr/bin/env python3
"""configs[2]-shaped measurement (not the bench.py headline): one seeded image-layer tar
(trivy_amd.configs.layer_tar) through the native ingest (tsg_layer_pack: tar walk +
Required + IsBinary + packing) and a GPU scan of the packed batch.

    python tools/layer_bench.py [GiB] [scans] [--emulate]
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
    emulate = "--emulate" in sys.argv  # (a CPU check of the harness: no GPU)
    argv = [a for a in sys.argv[1:] if a != "--emulate"]
    gib = float(argv[0]) if argv else 1.0
    scans = int(argv[1]) if len(argv) > 1 else 3
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
    ctx = S.GpuContext(an.scanner, 0, emulate=emulate)
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
    # configs[2] over W GPUs, rank by rank in this one process (each rank is its own process
    # on its own GPU in the deployment; here the slowest rank's time is what bounds them):
    # (a) every rank indexes the whole chain and packs only its byte run (tsg_layer_pack_shard);
    # (b) the distributed index (tsg_layer_range_*): each rank walks only its byte range, the
    #     exchange simulated in-process (layer_chain_step), then sync + dirs + pack.
    # Round 3 timed each world once and packed into fresh pageable memory: a pack faults its
    # whole output in (~44 k minor faults per quarter of a 1 GiB layer, about a third of its
    # time) and single calls stalled for 0.1-0.25 s now and then (host noise: the same fault
    # count, a different rank each time), which made the slowest rank non-monotonic.  Now
    # each world runs REPS times (median of the slowest rank), and (b) also packs into a
    # pinned slot of the context (tsg_layer_range_pack_slot), as the product ingest does,
    # whose memory is faulted in once.
    import resource
    import statistics

    def minflt():
        return resource.getrusage(resource.RUSAGE_SELF).ru_minflt

    REPS = 3
    shard = {}
    for world in (2, 4, 8):
        rows = []
        for _ in range(REPS):
            worst = 0.0
            for rank in range(world):
                t = time.perf_counter()
                W.NativeLayer(an.scanner, tar, rank=rank, world=world)
                worst = max(worst, time.perf_counter() - t)
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
            worst_r = worst_s = 0.0
            stage_r = stage_s = None
            prior, resync, faults = [], len(confirmed), 0
            for rank, g in enumerate(rngs):
                t = time.perf_counter()
                g.sync(st[1][rank])
                d = g.dirs()
                t1 = time.perf_counter()
                f0 = minflt()
                lay_r = g.pack(an.scanner, (), (), prior, "")
                t2 = time.perf_counter()
                faults = max(faults, minflt() - f0)
                del lay_r
                sl = W.SlotIngest.layer_range(ctx, g, (), (), prior, "")
                t3 = time.perf_counter()
                sl.release()
                tot = walk_t[rank] + (t1 - t) + (t2 - t1)
                tot_s = walk_t[rank] + (t1 - t) + (t3 - t2)
                if tot > worst_r:
                    worst_r, stage_r = tot, (walk_t[rank], t1 - t, t2 - t1)
                if tot_s > worst_s:
                    worst_s, stage_s = tot_s, (walk_t[rank], t1 - t, t3 - t2)
                prior = prior + d
            rows.append((worst, worst_r, worst_s, stage_r, stage_s, resync, faults))
        med = lambda k: statistics.median(r[k] for r in rows)  # noqa: E731
        mid = sorted(rows, key=lambda r: r[2])[len(rows) // 2]
        shard[str(world)] = {"slowest_rank_pack_s": round(med(0), 4),
                             "per_rank_ingest_GBps_of_tar": round(len(tar) / med(0) / 1e9, 2),
                             "range_index_slowest_rank_s": round(med(1), 4),
                             "range_index_per_rank_GBps_of_tar": round(len(tar) / med(1) / 1e9, 2),
                             "range_index_slot_slowest_rank_s": round(med(2), 4),
                             "range_index_slot_per_rank_GBps_of_tar": round(len(tar) / med(2) / 1e9, 2),
                             "slot_slowest_rank_stages_s": {"walk": round(mid[4][0], 4), "sync_dirs": round(mid[4][1], 4),
                                                            "pack_slot": round(mid[4][2], 4)},
                             "pageable_pack_minor_faults_max": int(med(6)),
                             "runs_slowest_rank_s": [[round(r[0], 4), round(r[1], 4), round(r[2], 4)] for r in rows],
                             "range_index_resyncs": rows[-1][5]}
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
