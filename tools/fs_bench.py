#!/usr/bin/env python3
"""BASELINE configs[0]: `trivy fs --scanners secret` over a seeded 200 MiB source tree,
end to end on one MI355X, with the exact CPU path timed beside it.

    python tools/fs_bench.py [--mib 200] [--dir DIR] [--threads 16] [--oracle-files 400]

Stages (each timed): native fs ingest (tsg_fs_pack: walk, `Required`, reads, IsBinary,
packing), the device scan of the packed batch (upload, K1, gates, K2, host resolution),
the analyzer sort and the Go-compatible JSON report.  The exact CPU path (the reference
algorithm restated, tsg_scan_cpu_batch) scans the same packed batch; its results must be
identical, and a sample of files is checked against the oracle.  Prints one JSON line.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=200)
    ap.add_argument("--dir", default="")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--oracle-files", type=int, default=40)
    args = ap.parse_args()
    from trivy_amd import analyzer as A
    from trivy_amd import configs
    from trivy_amd import report as R
    from trivy_amd import secret as S
    from trivy_amd import walker as W
    from tests.helpers import canon_secret

    tmp = args.dir or tempfile.mkdtemp(prefix="tsg_fs_")
    root = os.path.join(tmp, "tree")
    t0 = time.perf_counter()
    info = configs.source_tree(root, args.mib << 20, seed=0)
    gen_s = time.perf_counter() - t0
    an = A.SecretAnalyzer()
    an.Init("")
    sc = an.scanner
    ctx = S.GpuContext(sc, 0)
    W.analyze_fs(an, root, ctx=ctx)  # warm-up: first-use costs of the context
    t0 = time.perf_counter()
    fs = W.NativeFS(sc, root)
    t1 = time.perf_counter()
    res = sc.ScanBatch(fs.batch, ctx=ctx)
    t2 = time.perf_counter()
    # AnalysisResult.Sort reorders each secret's findings by (RuleID, StartLine) in place;
    # the parity checks below compare Scan's own order, so sort a copy
    secrets = A.sort_secrets([dict(r, Findings=list(r["Findings"])) for r in res if r["Findings"]])
    js = R.write_json(R.fs_report(root, R.secrets_to_results(R.apply_layers([{"Secrets": secrets}]))))
    t3 = time.perf_counter()
    ctx.close()
    nb = int(fs.batch.offsets[-1])
    c0 = time.perf_counter()
    cpu = sc.ScanBatch(fs.batch, nthreads=args.threads)
    cpu_s = time.perf_counter() - c0
    if cpu != res:
        bad = [i for i in range(len(res)) if cpu[i] != res[i]]
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "fs_bench_diff.json"), "w") as f:
            json.dump({"n_bad": len(bad), "cases": [
                {"path": fs.batch.path(i), "size": int(fs.batch.offsets[i + 1] - fs.batch.offsets[i]),
                 "device": canon_secret(res[i]), "cpu": canon_secret(cpu[i])} for i in bad[:20]]},
                f, indent=1, default=str)
        raise AssertionError("device results differ from the exact CPU path in %d files" % len(bad))
    from oracle import secret as O
    osc = O.NewScanner(None)
    step = max(1, fs.batch.nfiles // max(1, args.oracle_files))
    checked = 0
    for i in range(0, fs.batch.nfiles, step):
        c = bytes(fs.batch.data[int(fs.batch.offsets[i]):int(fs.batch.offsets[i + 1])])
        assert canon_secret(res[i]) == canon_secret(osc.Scan(fs.batch.path(i), c)), fs.batch.path(i)
        checked += 1
    line = {
        "workload": "trivy fs --scanners secret over a %d MiB seeded source tree (BASELINE configs[0]; "
                    "configs.source_tree)" % args.mib,
        "tree": info, "scanned_files": fs.batch.nfiles, "scanned_bytes": nb, "walked": fs.walked,
        "findings": sum(len(s["Findings"]) for s in secrets), "files_with_findings": len(secrets),
        "ingest_s": round(t1 - t0, 4), "ingest_GBps": round(info["bytes"] / (t1 - t0) / 1e9, 3),
        "scan_s": round(t2 - t1, 4), "scan_GBps": round(nb / (t2 - t1) / 1e9, 3),
        "report_s": round(t3 - t2, 4), "report_bytes": len(js),
        "e2e_s": round(t3 - t0, 4), "e2e_GBps": round(nb / (t3 - t0) / 1e9, 3),
        "cpu_exact": {"s": round(cpu_s, 3), "GBps": round(nb / cpu_s / 1e9, 4), "threads": args.threads,
                      "what": "tsg_scan_cpu_batch (scanner.go:341-416 restated) on the same packed batch"},
        "parity": {"device_vs_cpu_exact": "identical, %d files" % fs.batch.nfiles,
                   "device_vs_oracle_files": checked},
        "gen_s": round(gen_s, 2),
    }
    print(json.dumps(line), flush=True)
    if not args.dir:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
