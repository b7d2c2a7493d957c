"""K1F, the filter-and-verify K1 (trivy_amd/csrc/k1f.hpp), on the CPU: its algorithm with
the device's tables and bit logic (tsg_emulate_k1f) equals k1_reference -- the semantics of
Rule.MatchKeywords (pkg/fanal/secret/scanner.go:164-176) plus the chunk events K2 needs --
bit for bit, and leaving literals out of the filter (the adaptation) only removes their own
bits."""
import numpy as np
import pytest

from trivy_amd import configs, corpus
from trivy_amd import secret as S


@pytest.fixture(scope="module")
def builtin():
    return S.NewScanner(None)


def _eq(sc, batch, chunk, quiet=()):
    kw, ev = sc.k1_reference(batch, chunk)
    fk, fe, st = sc.k1f_emulate(batch, chunk, quiet)
    return kw, ev, fk, fe, st


@pytest.mark.parametrize("chunk", [16, 48, 256, 1024, 131072])
def test_emulation_equals_reference_corpus(builtin, chunk):
    batch, _ = corpus.make_corpus(2 << 20, seed=40 + chunk % 97, plants_per_mib=80)
    kw, ev, fk, fe, st = _eq(builtin, batch, chunk)
    assert np.array_equal(kw, fk)
    assert np.array_equal(ev, fe)
    assert st["arrivals"] > 0 and (ev & 1).any() and (ev & 2).any() and (ev >> 2).any()


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("chunk", [16, 48, 256])
def test_emulation_equals_reference_edges(builtin, seed, chunk):
    batch = corpus.k1_edge_batch(builtin.k1_literals(), seed)
    kw, ev, fk, fe, _ = _eq(builtin, batch, chunk)
    assert np.array_equal(kw, fk)
    assert np.array_equal(ev, fe)


def test_emulation_equals_reference_fold_runes(builtin):
    batch = corpus.fold_runes_batch(11, nbytes=1 << 20, plants=300, frac=0.3)
    kw, ev, fk, fe, _ = _eq(builtin, batch, 64)
    assert np.array_equal(kw, fk)
    assert np.array_equal(ev, fe)


def test_emulation_random_bytes(builtin):
    """Binary blobs with literals planted in random case."""
    rng = np.random.default_rng(5)
    lits = [s for s, _ in builtin.k1_literals()]
    args = []
    for i in range(300):
        b = bytearray(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes())
        for _ in range(int(rng.integers(0, 5))):
            s = lits[int(rng.integers(0, len(lits)))]
            p = int(rng.integers(0, len(b) + 1))
            b[p:p] = bytes(c - 32 if 97 <= c <= 122 and rng.random() < 0.5 else c for c in s)
        args.append(S.ScanArgs("b/%d" % i, bytes(b)))
    batch = S.Batch.from_args(args)
    kw, ev, fk, fe, _ = _eq(builtin, batch, 256)
    assert np.array_equal(kw, fk)
    assert np.array_equal(ev, fe)


def test_quiet_literals_remove_only_their_bits(builtin):
    """The adaptation's hot literals leave the filter: their keywords' bits may vanish (the
    host then checks them exactly), every other bit stays, nothing is added."""
    lits = builtin.k1_literals()
    nkw = builtin.info()["n_keywords"]
    hot = [b"sk", b"lob", b"key", b"live_", b"account", b"sg.", b"linear", b"pk.", b"-----"]
    quiet = [i for i, (s, _) in enumerate(lits) if s in hot]
    assert len(quiet) == len(hot)
    batch, _ = corpus.make_corpus(4 << 20, seed=9)
    kw, ev, fk, fe, st = _eq(builtin, batch, 256, quiet)
    assert np.all((fk & ~kw) == 0) and np.all((fe & ~ev) == 0)
    keep = np.zeros(kw.shape[1], dtype=np.uint32)
    for k in range(nkw):
        if k not in quiet:
            keep[k // 32] |= np.uint32(1 << (k % 32))
    assert np.array_equal(kw & keep, fk & keep)
    assert st["records"] == len(lits) - len(quiet)
    # the static buckets keep the words listed for verification rare on this corpus
    assert st["groups"] < int(batch.offsets[-1]) / 1024 * 8


def test_k1f_applies_per_config():
    """configs[4] (allow rules, exclude blocks) and the 1,000-rule set of configs[3] run K1F
    with k1_reference's semantics.  configs[3]'s K1 keeps a slot per keyword id: the 783
    keywords K1X takes are never-matching slots (dfa.hpp never_literal), so K1F holds its
    121 real literals (it declined the 904 slots before round 6)."""
    for name, doc in (("allow-exclude", configs.allow_exclude_doc()),
                      ("user1000", configs.user_rules_doc(1000, seed=4))):
        sc = S.NewScanner(S.config_from_dict(doc))
        batch = corpus.k1_edge_batch(sc.k1_literals(), 4, nfiles=200)
        kw, ev, fk, fe, st = _eq(sc, batch, 256)
        assert np.array_equal(kw, fk)
        assert np.array_equal(ev, fe)
        if name == "user1000":
            assert st["records"] == 121


def test_sample_priced_filter(builtin):
    """The adaptation's rebuild prices windows and buckets by their counts in a sample of
    the data: same bits as k1_reference (for the literals it keeps), and far fewer words
    listed for verification than the text-model buckets on the same corpus."""
    lits = builtin.k1_literals()
    hot = [b"sk", b"lob", b"key", b"live_", b"account", b"sg.", b"linear", b"pk.", b"-----"]
    quiet = [i for i, (s, _) in enumerate(lits) if s in hot]
    batch, _ = corpus.make_corpus(8 << 20, seed=13, plants_per_mib=20)
    kw, ev = builtin.k1_reference(batch, 256)
    fk0, fe0, st0 = builtin.k1f_emulate(batch, 256, quiet)
    fk, fe, st = builtin.k1f_emulate(batch, 256, quiet, sample_kib=1024)
    assert np.array_equal(fk, fk0) and np.array_equal(fe, fe0)
    assert np.all((fk & ~kw) == 0) and np.all((fe & ~ev) == 0)
    assert st["arrivals"] == st0["arrivals"]
    assert st["groups"] * 5 < st0["groups"]


@pytest.mark.parametrize("chunk", [16, 256])
def test_sample_priced_filter_edges(builtin, chunk):
    """Sample-priced buckets (sampled from the edge batch itself) keep the exact semantics."""
    batch = corpus.k1_edge_batch(builtin.k1_literals(), 21)
    kw, ev = builtin.k1_reference(batch, chunk)
    fk, fe, _ = builtin.k1f_emulate(batch, chunk, sample_kib=64)
    assert np.array_equal(kw, fk)
    assert np.array_equal(ev, fe)
