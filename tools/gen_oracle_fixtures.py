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

Oracle samples (the smaller per-test expectations of the GPU tests and smoke(), so that no
code under oracle/ runs on the GPU box): SAMPLES names a seeded input per test (the files a
test compares with the oracle); their canonical results are stored under
tests/golden/oracle_small/<name>.json.gz with a sha256 of the inputs, and `sample_expect`
hands them to the test after checking that the regenerated inputs match.

    python tools/gen_oracle_fixtures.py --samples [name ...]   (default: every sample)
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


def _builtin_batch(mib_k, seed, plants, every=1):
    from trivy_amd import corpus
    b, _ = corpus.make_corpus(mib_k << 10, seed=seed, plants_per_mib=plants)
    return None, _batch_args(b, every)


def _batch_args(b, every=1):
    from trivy_amd import secret as S
    return [S.ScanArgs(b.path(i), bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])]))
            for i in range(0, b.nfiles, every)]


def _fold():
    from trivy_amd import corpus
    return None, _batch_args(corpus.fold_runes_batch(3, nbytes=128 << 10, plants=400, frac=0.6))


def _tree(scratch, mib, seed, every):
    from trivy_amd import analyzer as A
    from trivy_amd import configs
    from trivy_amd import walker as W
    root = os.path.join(scratch, "tree")
    configs.source_tree(root, mib << 20, seed=seed)
    an = A.SecretAnalyzer()
    an.Init("")
    return None, _batch_args(W.NativeFS(an.scanner, root).batch, every)


def _layer(mib, seed, every, binary_frac=0.05, big=(), skip_dirs=()):
    from trivy_amd import analyzer as A
    from trivy_amd import configs
    from trivy_amd import walker as W
    an = A.SecretAnalyzer()
    an.Init("")
    tar = configs.layer_tar(mib << 20, seed=seed, binary_frac=binary_frac, big=big)
    return None, _batch_args(W.NativeLayer(an.scanner, tar, skip_dirs=skip_dirs).batch, every)


def _user1000():
    from trivy_amd import configs
    doc = configs.user_rules_doc(1000, seed=4)
    return doc, configs.mixed_batch(doc, 256 << 10, seed=61, plants_per_file=0.6)


def _allow_exclude():
    from trivy_amd import analyzer as A
    from trivy_amd import configs
    doc = configs.allow_exclude_doc()
    args = configs.mixed_batch(doc, 256 << 10, seed=62, plants_per_file=0.5, binary_frac=0.3)
    return doc, [a for a in args if not A.IsBinary(a.Content, len(a.Content))]


# name -> f(scratch dir) -> (rules config doc or None, [ScanArgs]): the files each GPU test
# (and smoke()) compares with the oracle; the tests build the same inputs and take the
# expected results from tests/golden/oracle_small/ (sample_expect)
SAMPLES = {
    "smoke": lambda d: _builtin_batch(96, 11, 400),                    # __graft_entry__.smoke
    "corpus": lambda d: _builtin_batch(256, 7, 300),                   # test_corpus_vs_oracle
    "fold_runes": lambda d: _fold(),                                   # test_fold_runes_gpu_vs_oracle
    "config0_tree": lambda d: _tree(d, 8, 0, 32),                      # test_source_tree_config0_gpu
    "multi": lambda d: _builtin_batch(24 << 10, 77, 40, 97),           # test_multi_two_contexts_one_device_gpu
    "slot_fs": lambda d: _tree(d, 6, 3, 41),                           # test_slot_ingest_gpu
    "slot_layer": lambda d: _layer(6, 5, 41, 0.1),                     # test_slot_ingest_gpu
    "big_layer": lambda d: _layer(2, 12, 1, 0.0, big=(3 << 20, (1 << 20) + 4096)),  # test_file_larger_than_slot_gpu
    "layer36": lambda d: _layer(12, 36, 1, skip_dirs=["/deep"]),        # test_native_layer_gpu_vs_oracle
    "two_rank_layer": lambda d: _layer(6, 21, 1),                      # test_two_ranks_layer_gpu
    "user1000": lambda d: _user1000(),                                 # test_user_rules_1000_gpu_vs_oracle
    "allow_exclude": lambda d: _allow_exclude(),                       # test_allow_exclude_binary_gpu_vs_oracle
}
SMALL = os.path.join(ROOT, "tests", "golden", "oracle_small")


def sample_expect(name, args):
    """The oracle's canonical results for sample `name`, after checking that `args` (the
    test's own inputs, in its order) are the fixture's."""
    with gzip.open(os.path.join(SMALL, name + ".json.gz"), "rt", encoding="utf-8") as f:
        rec = json.load(f)
    assert digest(args) == rec["sha256"], "sample %s: the inputs differ from the fixture's" % name
    return rec["secrets"]


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


def _run_oracle(name, doc, args, procs):
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
    return want


def samples(names, procs):
    import tempfile
    os.makedirs(SMALL, exist_ok=True)
    for name in names:
        t0 = time.time()
        with tempfile.TemporaryDirectory() as d:
            doc, args = SAMPLES[name](d)
        want = _run_oracle(name, doc, args, procs)
        rec = {"sample": name, "files": len(args), "bytes": sum(len(a.Content) for a in args),
               "sha256": digest(args), "findings": sum(len(w["Findings"] or []) for w in want if w),
               "generator": "tools/gen_oracle_fixtures.py --samples (oracle/secret.py)", "secrets": want}
        with gzip.open(os.path.join(SMALL, name + ".json.gz"), "wt", encoding="utf-8") as f:
            json.dump(rec, f, separators=(",", ":"))
        print("%s: %d files, %d findings, oracle %.0f s" % (name, len(args), rec["findings"], time.time() - t0),
              flush=True)


def main():
    procs = int(os.environ.get("ORACLE_PROCS", str(os.cpu_count() or 4)))
    if sys.argv[1:2] == ["--samples"]:
        samples(sys.argv[2:] or list(SAMPLES), procs)
        return
    names = sys.argv[1:] or list(WORKLOADS)
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
