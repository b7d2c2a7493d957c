"""The product's exact CPU path (libtrivy_secret.so) against the reference's own fixtures
and against the oracle.  No GPU needed."""
import os

import pytest

from tests.conftest import GOLDEN
from tests.helpers import canon_secret, reference_cases
from trivy_amd import analyzer as A
from trivy_amd import secret as S

CASES = reference_cases()
SDIR = os.path.join(GOLDEN, "reference", "secret")
ADIR = os.path.join(GOLDEN, "reference", "analyzer")


@pytest.fixture
def in_dir():
    old = os.getcwd()
    yield lambda d: os.chdir(d)
    os.chdir(old)


@pytest.mark.parametrize("case", CASES["scanner_cases"], ids=lambda c: c["name"])
def test_scanner_case_cpu(case, in_dir):
    in_dir(SDIR)
    content = open(case["input"], "rb").read()
    s = S.NewScanner(S.ParseConfig(case["config"]))
    got = s.Scan(S.ScanArgs(case["input"], content))
    assert canon_secret(got) == case["want"]


@pytest.mark.parametrize("case", CASES["scanner_cases"], ids=lambda c: c["name"])
@pytest.mark.parametrize("chunk", [16, 64, 256])
def test_scanner_case_emulated_kernels(case, chunk, in_dir):
    """The GPU algorithm (K1/K2 chunking, candidate windows) emulated on the CPU."""
    in_dir(SDIR)
    content = open(case["input"], "rb").read()
    s = S.NewScanner(S.ParseConfig(case["config"]))
    got = s.ScanBatch([S.ScanArgs(case["input"], content)], emulate_chunk=chunk)[0]
    assert canon_secret(got) == case["want"]


@pytest.mark.parametrize("case", CASES["analyzer_cases"], ids=lambda c: c["name"])
def test_analyzer_case(case, in_dir):
    in_dir(ADIR)
    a = A.SecretAnalyzer()
    a.Init(case["config"])
    content = open(case["input"], "rb").read()
    got = a.Analyze(A.AnalysisInput(Dir=case["dir"], FilePath=case["input"], Content=content))
    if case["want"] is None:
        assert got is None
    else:
        assert [canon_secret(x) for x in got["Secrets"]] == case["want"]["Secrets"]


@pytest.mark.parametrize("case", CASES["required_cases"], ids=lambda c: c["name"])
def test_required_case(case, in_dir):
    in_dir(ADIR)
    a = A.SecretAnalyzer()
    a.Init("")
    assert a.Required(case["input"], os.path.getsize(case["input"])) == case["want"]
