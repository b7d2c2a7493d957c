#!/usr/bin/env python3
"""Device vs the independent oracle (oracle/secret.py, a Python restatement of scanner.go
that shares no code with the product's resolver) on EVERY file of seeded corpora larger
than the test suite's: the product's GPU path (HIP kernels + host resolution) must equal the
oracle file by file.  Test infrastructure (it imports oracle/), run as its own process on
the GPU box, not collected by pytest (profiles/r04/oracle_bulk/):

    python tests/oracle_bulk.py OUT.json [configs1_MiB=16] [configs3_MiB=1] [configs4_MiB=4]

The oracle runs first, in a pool of forked workers, before this process touches the GPU
(no process is forked or exec'd after HIP is initialised); then the device scans.
"""
import json
import os
import sys
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

_JOB = {}


def _oracle_chunk(idx):
    from oracle import secret as O
    from tests.helpers import canon_secret
    osc = O.NewScanner(O.config_from_dict(_JOB["doc"]))
    return [canon_secret(osc.Scan(_JOB["args"][i].FilePath, _JOB["args"][i].Content)) for i in idx]


def _oracle_pair(idx):
    return idx, _oracle_chunk(idx)


def _workload(name, mib):
    from trivy_amd import configs, corpus
    from trivy_amd import secret as S
    import numpy as np
    if name == "configs1":
        b, _ = corpus.make_corpus(mib << 20, seed=11, plants_per_mib=8.0)
        args = [S.ScanArgs(b.path(i), bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])]))
                for i in range(b.nfiles)]
        return {}, args
    if name == "configs3":
        doc = configs.user_rules_doc(1000, seed=4)
        return doc, configs.mixed_batch(doc, mib << 20, seed=31, plants_per_file=0.6)
    doc = configs.allow_exclude_doc()
    from trivy_amd import analyzer as A
    args = configs.mixed_batch(doc, mib << 20, seed=32, plants_per_file=0.5, binary_frac=0.3)
    return doc, [a for a in args if not A.IsBinary(a.Content, len(a.Content))]


def main():
    out = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2:5]] + [16, 1, 4][len(sys.argv[2:5]):]
    procs = int(os.environ.get("ORACLE_PROCS", "16"))
    work = []
    for name, mib in zip(("configs1", "configs3", "configs4"), sizes):
        if mib <= 0:
            continue
        doc, args = _workload(name, mib)
        _JOB.update(doc=doc, args=args)
        t0 = time.time()
        idx = list(range(len(args)))
        nparts = max(procs, min(len(args), 16 * procs))
        parts = [idx[k::nparts] for k in range(nparts)]
        want = [None] * len(args)
        last = time.time()
        with get_context("fork").Pool(procs) as pool:
            for done, (part, r) in enumerate(pool.imap_unordered(_oracle_pair, parts), 1):
                for i, v in zip(part, r):
                    want[i] = v
                if time.time() - last > 20:  # progress (a silent run looks hung on the box)
                    print("  %s: %d / %d parts" % (name, done, len(parts)), flush=True)
                    last = time.time()
        work.append((name, mib, doc, args, want, time.time() - t0))
        print("%s: oracle over %d files (%d MiB) in %.0f s" % (name, len(args), mib, time.time() - t0), flush=True)
    # the GPU only from here on
    from tests.helpers import canon_secret
    from trivy_amd import secret as S
    report = {"what": __doc__.split("\n\n")[0], "runs": []}
    ok = True
    for name, mib, doc, args, want, osec in work:
        sc = S.NewScanner(S.config_from_dict(doc)) if doc else S.NewScanner(None)
        # (ORACLE_EMULATE=1: the kernels emulated on the CPU, a dry run of this script)
        got = (sc.ScanBatch(args, emulate_chunk=256) if os.environ.get("ORACLE_EMULATE")
               else sc.ScanBatch(args, device=0))
        bad = [a.FilePath for a, g, w in zip(args, got, want) if canon_secret(g) != w]
        nf = sum(len(w["Findings"] or []) for w in want if w)
        report["runs"].append({"config": name, "MiB": mib, "files": len(args),
                               "bytes": sum(len(a.Content) for a in args), "findings": nf,
                               "mismatched_files": bad[:20], "n_mismatched": len(bad),
                               "oracle_s": round(osec, 1), "rules": len(sc.Rules)})
        ok = ok and not bad
        print("%s: %d files, %d findings, %d mismatched" % (name, len(args), nf, len(bad)), flush=True)
    report["equal"] = ok
    with open(out, "w") as f:
        json.dump(report, f, indent=1)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
