"""configs[3] / configs[4] parity on the device: HIP kernels + host resolution through the
C ABI, file by file against the oracle (oracle/secret.py, a restatement of scanner.go, through
its committed results in tests/golden/oracle_small/) and
against the exact CPU path on larger batches.  No reference fixture covers these rule
sets; the oracle is pinned by the reference fixtures (test_oracle_reference.py)."""
import pytest

from tests.helpers import canon_secret
from tools.gen_oracle_fixtures import sample_expect
from trivy_amd import analyzer as A
from trivy_amd import configs
from trivy_amd import secret as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def user1000():
    doc = configs.user_rules_doc(1000, seed=4)
    return doc, S.NewScanner(S.config_from_dict(doc))


def _vs_oracle(name, args, got):
    """got == the oracle's results for sample `name` (oracle/secret.py over the same seeded
    inputs, committed under tests/golden/oracle_small/ by tools/gen_oracle_fixtures.py)."""
    n = 0
    want = sample_expect(name, args)
    assert len(want) == len(got)
    for a, g, w in zip(args, got, want):
        assert canon_secret(g) == w, a.FilePath
        n += len(w["Findings"] or [])
    return n


def test_user_rules_1000_compile(user1000):
    """configs[3] at its stated size: 1,000 user rules + 83 builtins compile into a plan."""
    _, sc = user1000
    info = sc.info()
    assert info["n_rules"] == 1083 and info["n_groups"] > 0


def _k1_vs_reference(sc, b, chunks=(64, 256)):
    import numpy as np
    for chunk in chunks:
        ctx = S.GpuContext(sc, 0, chunk_bytes=chunk, adapt_mib=0xFFFFFFFF)
        ctx.upload(b)
        ctx.kernels()
        kw, ev = ctx.k1_output(chunk)
        ctx.close()
        rkw, rev = sc.k1_reference(b, chunk)
        assert np.array_equal(kw, rkw)
        assert np.array_equal(ev, rev)


@pytest.mark.parametrize("step", [None, "1", "2", "4"])
def test_user_rules_1000_k1_vs_reference(step, knob):
    """configs[3]'s keywords and anchors do not fit K1's automaton: the builtin rules' and
    the short ones stay, the rest go to the hashed prefilter (K1X), which samples a window
    every `step` bytes (None: the plan's choice).  K1 + K1X keyword bits and chunk events
    == k1_reference."""
    if step:
        knob("x_step", step)
    doc = configs.user_rules_doc(1000, seed=4)
    sc = S.NewScanner(S.config_from_dict(doc))
    assert sc.info()["k1x_literals"] > 800
    _k1_vs_reference(sc, S.Batch.from_args(configs.mixed_batch(doc, 1 << 20, seed=65, plants_per_file=0.8)))


@pytest.mark.parametrize("step", ["1", "2", "4"])
def test_k1x_every_alignment(step, knob):
    """K1X literals at every byte alignment, periodic literals (one 4-gram at several
    offsets), overlapping occurrences, occurrences straddling file boundaries and ending at
    the batch's last byte: keyword bits and events == k1_reference."""
    knob("x_step", step)
    doc = configs.user_rules_doc(1000, seed=4)
    extra = ["aaaaaaaaq", "qzqzqzqzqz", "Mixed-Case-Key", "zzzzzzzz"]
    for i, k in enumerate(extra):
        doc["rules"].append({"id": "extra-%d" % i, "category": "user", "title": "extra", "severity": "LOW",
                             "regex": r"(?i)%s(?P<secret>[0-9a-z]{8})" % k.lower().replace("-", r"\-"),
                             "keywords": [k]})
    sc = S.NewScanner(S.config_from_dict(doc))
    files = []
    for off in range(20):
        for k in extra:
            files.append(("f%d_%s" % (off, k), b"." * off + k.upper().encode() + b"0123abcd" + b"aaaa" * (off % 3)))
    files.append(("periodic", b"aaaaaaaaaaaaaaaqzqzqzqzqzqzqzqzq" * 9 + b"zzzzzzzzzzzzzzzzzzzzz"))
    # a literal split across two files, and one ending at the batch's last byte
    files.append(("split_a", b"xxxxxxxxxxxxxMixed-Ca"))
    files.append(("split_b", b"se-Key00000000 zzzz"))
    files.append(("last", b"........................zzzzzzzz"))
    b = S.Batch.from_args([S.ScanArgs(FilePath=n, Content=c) for n, c in files])
    _k1_vs_reference(sc, b, chunks=(16, 64))


def test_user_rules_1000_gpu_vs_oracle(user1000):
    doc, sc = user1000
    args = configs.mixed_batch(doc, 256 << 10, seed=61, plants_per_file=0.6)
    got = sc.ScanBatch(args, device=0)
    assert _vs_oracle("user1000", args, got) > 10


def test_user_rules_1000_gpu_vs_exact(user1000):
    doc, sc = user1000
    b = S.Batch.from_args(configs.mixed_batch(doc, 2 << 20, seed=63))
    want = sc.ScanBatch(b, nthreads=16)
    assert sc.ScanBatch(b, device=0) == want
    assert sum(len(x["Findings"] or []) for x in want) > 10


def test_allow_exclude_binary_gpu_vs_oracle():
    doc = configs.allow_exclude_doc()
    sc = S.NewScanner(S.config_from_dict(doc))
    args = configs.mixed_batch(doc, 256 << 10, seed=62, plants_per_file=0.5, binary_frac=0.3)
    args = [a for a in args if not A.IsBinary(a.Content, len(a.Content))]
    got = sc.ScanBatch(args, device=0)
    assert _vs_oracle("allow_exclude", args, got) > 5


def test_allow_exclude_binary_gpu_vs_exact():
    doc = configs.allow_exclude_doc()
    sc = S.NewScanner(S.config_from_dict(doc))
    args = configs.mixed_batch(doc, 2 << 20, seed=64, plants_per_file=0.5, binary_frac=0.3)
    args = [a for a in args if not A.IsBinary(a.Content, len(a.Content))]
    b = S.Batch.from_args(args)
    want = sc.ScanBatch(b, nthreads=16)
    assert sc.ScanBatch(b, device=0) == want
    assert sum(len(x["Findings"] or []) for x in want) > 5


def test_hostonly_rule_gpu_vs_exact():
    """A rule no DFA fits (3,000 12-letter words in one alternation: no counted repetition
    to relax, one top-level atom) is resolved on the host over every file, so the outputs
    kernel hands back every file's keyword row (its sparse form covers only files with
    candidates or flags).  Device == exact CPU path, with the word planted in some files."""
    import numpy as np
    rng = np.random.default_rng(7)
    words = ["".join(rng.choice(list("abcdefghijklmnopqrstuvwxyz"), size=12)) for _ in range(3000)]
    doc = {"rules": [{"id": "many-words", "category": "custom", "title": "many words", "severity": "LOW",
                      "regex": "(?P<secret>(?:" + "|".join(words) + "))"}]}
    sc = S.NewScanner(S.config_from_dict(doc))
    assert sc.info()["n_hostonly"] == 1
    args = configs.mixed_batch(doc, 1 << 20, seed=66, plants_per_file=0.3)
    args += [S.ScanArgs("w/%d.txt" % i, ("x = %s\n" % words[i * 7]).encode()) for i in range(40)]
    b = S.Batch.from_args(args)
    want = sc.ScanBatch(b, nthreads=16)
    assert sc.ScanBatch(b, device=0) == want
    assert sum(1 for x in want if any(f["RuleID"] == "many-words" for f in x["Findings"] or [])) >= 40


def test_k1x_list_overflow_inline_verify():
    """Every 16-byte word of a 2 MiB batch holds a K1X literal (a periodic one, repeated):
    the blocks' list slices overflow and the rest of the hits are verified inline in
    k1x_kernel.  Keyword bits and events == k1_reference; the inline path ran."""
    doc = configs.user_rules_doc(1000, seed=4)
    doc["rules"].append({"id": "periodic", "category": "user", "title": "periodic", "severity": "LOW",
                         "regex": r"qzqzqzqzqz(?P<secret>[0-9]{4})", "keywords": ["qzqzqzqzqz"]})
    sc = S.NewScanner(S.config_from_dict(doc))
    files = [S.ScanArgs("p/%d.txt" % i, b"qz" * (16 << 10) + b"0123\n") for i in range(64)]
    b = S.Batch.from_args(files)
    _k1_vs_reference(sc, b, chunks=(256,))
    ctx = S.GpuContext(sc, 0, chunk_bytes=256, adapt_mib=0xFFFFFFFF)
    ctx.upload(b)
    ctx.kernels()
    st = ctx.stats()
    ctx.close()
    assert st["k1x_inline"] > 0 and st["k1x_records"] > 0
