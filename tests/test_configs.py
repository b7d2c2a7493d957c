"""BASELINE configs[3] and configs[4] as parity cases: large user rule
sets (keyword-less rules, unbounded rules, DFA state blow-up, keywords left out of the
K1 automaton when it outgrows its LDS budget) and allow rules / exclude blocks / binary
blobs.  The GPU algorithm (emulated here, on the device in test_gpu_configs) must give
exactly the findings of the exact CPU path (Scanner.Scan, scanner.go:341-416).  No
reference fixture covers these rule sets: the expected side is the exact CPU path, which
the reference fixtures pin (test_cpu_reference.py)."""
import numpy as np
import pytest

from trivy_amd import analyzer as A
from trivy_amd import configs
from trivy_amd import secret as S


@pytest.fixture(scope="module")
def user100():
    doc = configs.user_rules_doc(100, seed=4)
    return doc, S.NewScanner(S.config_from_dict(doc))


def test_user_rules_plan_degrades_not_fails(user100):
    """183 rules: the K1 automaton would exceed its LDS budget; literals move to the hashed
    prefilter (K1X) instead of failing the rule-set compile (the reference has no such
    limit), and no keyword becomes unknown."""
    _, sc = user100
    info = sc.info()
    assert info["n_rules"] == 183 and info["kw_states"] > 0 and info["k1x_literals"] > 50


def test_k1x_reference_matches_bruteforce(user100):
    """k1_reference's keyword bits for a K1X rule set (most keywords hashed) == a brute-force
    search of every keyword in every ASCII-lowercased file.  Keyword ids follow the plan's
    numbering: first appearance over the rules' keywords (plan.cpp build_plan)."""
    doc, sc = user100
    b = S.Batch.from_args(configs.mixed_batch(doc, 64 << 10, seed=77, plants_per_file=0.9))
    kw, _ = sc.k1_reference(b, 256)
    ids = {}
    for r in sc.Rules:
        ks = [k.lower() for k in (r.Keywords or [])]
        if not all(k.isascii() for k in ks):
            continue
        for k in ks:
            ids.setdefault(k, len(ids))
    hits = 0
    for f in range(b.nfiles):
        low = bytes(b.data[int(b.offsets[f]):int(b.offsets[f + 1])]).lower()
        for k, i in ids.items():
            want = k.encode() in low
            got = bool((int(kw[f, i // 32]) >> (i % 32)) & 1)
            assert got == want, (f, k)
            hits += want
    assert hits > 20


def test_k1x_split_per_step(knob):
    """The x_step knob: 4 keeps every literal under 7 bytes in K1 (the largest automaton),
    1 hashes down to 4 bytes; the default is the widest step whose K1 table is packed
    (<= 64 KiB of u16 rows).  An unsupported step is an argument error."""
    from trivy_amd import _native as N
    doc = configs.user_rules_doc(1000, seed=4)
    info = {}
    for st in (None, "4", "2", "1"):
        if st:
            knob("x_step", st)
        info[st] = S.NewScanner(S.config_from_dict(doc)).info()
    assert info["4"]["kw_states"] > info["2"]["kw_states"] >= info["1"]["kw_states"]
    assert info["4"]["k1x_literals"] < info["2"]["k1x_literals"] <= info["1"]["k1x_literals"]
    assert info[None]["kw_states"] * info[None]["kw_classes"] * 2 <= 65536
    assert info[None] == info["2"]
    with pytest.raises(Exception):
        N.knob("x_step", "3")


@pytest.mark.parametrize("chunk", [64, 256])
def test_user_rules_emulation_vs_exact(user100, chunk):
    doc, sc = user100
    b = S.Batch.from_args(configs.mixed_batch(doc, 192 << 10, seed=40 + chunk))
    want = sc.ScanBatch(b, nthreads=8)
    assert sc.ScanBatch(b, emulate_chunk=chunk) == want
    assert sum(len(x["Findings"] or []) for x in want) > 10


def test_allow_exclude_binary_emulation_vs_exact():
    doc = configs.allow_exclude_doc()
    sc = S.NewScanner(S.config_from_dict(doc))
    args = configs.mixed_batch(doc, 256 << 10, seed=51, plants_per_file=0.5, binary_frac=0.3)
    # analyzer gate first (utils.IsBinary, secret.go:78-110), as the analyzer does
    args = [a for a in args if not A.IsBinary(a.Content, len(a.Content))]
    b = S.Batch.from_args(args)
    want = sc.ScanBatch(b, nthreads=8)
    assert sc.ScanBatch(b, emulate_chunk=256) == want
    n = sum(len(x["Findings"] or []) for x in want)
    assert n > 5
    assert any("blob/" in x.get("FilePath", "") for x in want if x["Findings"])


def _vs_oracle(doc, args, got):
    from oracle import secret as O
    from tests.helpers import canon_secret
    osc = O.NewScanner(O.config_from_dict(doc))
    n = 0
    for a, g in zip(args, got):
        want = canon_secret(osc.Scan(a.FilePath, a.Content))
        assert canon_secret(g) == want, a.FilePath
        n += len(want["Findings"] or [])
    return n


@pytest.fixture(scope="module")
def user1000():
    doc = configs.user_rules_doc(1000, seed=4)
    return doc, S.NewScanner(S.config_from_dict(doc))


def test_user_rules_1000_emulation_vs_oracle(user1000):
    """configs[3] at its stated size (1,000 user rules): the GPU algorithm, emulated,
    file by file against the oracle (not the product's own CPU path)."""
    doc, sc = user1000
    args = configs.mixed_batch(doc, 128 << 10, seed=71, plants_per_file=0.6)
    got = sc.ScanBatch(args, emulate_chunk=256)
    assert _vs_oracle(doc, args, got) > 10


def test_allow_exclude_binary_emulation_vs_oracle():
    doc = configs.allow_exclude_doc()
    sc = S.NewScanner(S.config_from_dict(doc))
    args = configs.mixed_batch(doc, 192 << 10, seed=72, plants_per_file=0.5, binary_frac=0.3)
    args = [a for a in args if not A.IsBinary(a.Content, len(a.Content))]
    got = sc.ScanBatch(args, emulate_chunk=64)
    assert _vs_oracle(doc, args, got) > 5


def test_group_caps(knob):
    """K2 rule-group caps: the builtin rules (83, under 256) get groups of up to 2,048 states
    / 64 KiB by default; the knobs set other caps, and a table cap past the u16 row offsets'
    64 KiB is an argument error.  Every group fits its caps."""
    from trivy_amd import _native as N
    default = S.NewScanner(None).info()
    knob("group_states", "1024")
    knob("group_table_kib", "48")
    small = S.NewScanner(None).info()
    assert default["n_groups"] < small["n_groups"]
    assert small["max_group_states"] <= 1024 < default["max_group_states"] <= 2048
    with pytest.raises(Exception):
        N.knob("group_table_kib", "65")
