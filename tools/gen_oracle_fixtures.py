#!/usr/bin/env python3
"""Oracle fixtures at size (SURVEY.md §8c's golden-vector plan): the independent oracle
(oracle/secret.py, a Python restatement of scanner.go sharing no code with the product's
resolver) run over seeded corpora of BASELINE configs[1] (16 MiB, builtin rules),
configs[3] (2 MiB, 1,000 user rules) and configs[4] (4 MiB, allow rules + exclude blocks,
binary blobs dropped by IsBinary).  Stored per workload under tests/golden/oracle_bulk/:
the seeds and sizes, a sha256 of the regenerated inputs, and every file's canonical
types.Secret.  tests/test_gpu_oracle_fixtures.py regenerates the corpora from the seeds,
scans them on the device and compares file by file -- the oracle itself never runs on the
GPU box (it scans 15-60 KB/s).

    python tools/gen_oracle_fixtures.py [workload ...]   (default: all three)
"""
import gzip
import hashlib
import json
import os
import sys
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "oracle_bulk")

# name -> (config, MiB, seed); tests/test_gpu_oracle_fixtures.py regenerates from these
WORKLOADS = {"configs1": ("builtin", 16, 11), "configs3": ("user1000", 2, 31), "configs4": ("allow-exclude", 4, 32)}

_JOB = {}


def workload(name):
    """(rules config doc or None, [ScanArgs]) of a fixture workload, from its seed."""
    from trivy_amd import analyzer as A
    from trivy_amd import configs, corpus
    from trivy_amd import secret as S
    kind, mib, seed = WORKLOADS[name]
    if kind == "builtin":
        b, _ = corpus.make_corpus(mib << 20, seed=seed, plants_per_mib=40.0)
        return None, [S.ScanArgs(b.path(i), bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])]))
                      for i in range(b.nfiles)]
    if kind == "user1000":
        doc = configs.user_rules_doc(1000, seed=4)
        return doc, configs.mixed_batch(doc, mib << 20, seed=seed, plants_per_file=0.6)
    doc = configs.allow_exclude_doc()
    args = configs.mixed_batch(doc, mib << 20, seed=seed, plants_per_file=0.5, binary_frac=0.3)
    return doc, [a for a in args if not A.IsBinary(a.Content, len(a.Content))]


def digest(args):
    h = hashlib.sha256()
    for a in args:
        h.update(a.FilePath.encode("utf-8", "surrogateescape") + b"\0")
        h.update(len(a.Content).to_bytes(8, "little") + a.Content)
    return h.hexdigest()


def _oracle_pair(idx):
    from oracle import secret as O
    from tests.helpers import canon_secret
    osc = O.NewScanner(O.config_from_dict(_JOB["doc"]) if _JOB["doc"] else None)
    return idx, [canon_secret(osc.Scan(_JOB["args"][i].FilePath, _JOB["args"][i].Content)) for i in idx]


def main():
    names = sys.argv[1:] or list(WORKLOADS)
    procs = int(os.environ.get("ORACLE_PROCS", str(os.cpu_count() or 4)))
    os.makedirs(OUT, exist_ok=True)
    for name in names:
        doc, args = workload(name)
        _JOB.update(doc=doc, args=args)
        t0 = time.time()
        idx = list(range(len(args)))
        nparts = min(len(args), 16 * procs)
        parts = [idx[k::nparts] for k in range(nparts)]
        want = [None] * len(args)
        with get_context("fork").Pool(procs) as pool:
            for done, (part, r) in enumerate(pool.imap_unordered(_oracle_pair, parts), 1):
                for i, v in zip(part, r):
                    want[i] = v
                if done % 16 == 0:
                    print("  %s: %d / %d parts, %.0f s" % (name, done, len(parts), time.time() - t0), flush=True)
        kind, mib, seed = WORKLOADS[name]
        rec = {"workload": name, "rules": kind, "MiB": mib, "seed": seed, "files": len(args),
               "bytes": sum(len(a.Content) for a in args), "sha256": digest(args),
               "findings": sum(len(w["Findings"] or []) for w in want if w),
               "generator": "tools/gen_oracle_fixtures.py (oracle/secret.py)",
               "secrets": want}
        with gzip.open(os.path.join(OUT, name + ".json.gz"), "wt", encoding="utf-8") as f:
            json.dump(rec, f, separators=(",", ":"))
        print("%s: %d files, %d findings, oracle %.0f s" % (name, len(args), rec["findings"], time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
