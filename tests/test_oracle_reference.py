"""Pin the CPU oracle against every fixture the reference's own tests hold.

scanner_test.go:529-746 (26 Scan cases), analyzer secret_test.go:105-223
(5 Analyze + 5 Required cases) and integration/testdata/secrets.json.golden.
"""
import os

import pytest

from oracle import secret as O
from tests.conftest import GOLDEN
from tests.helpers import canon_secret, reference_cases

CASES = reference_cases()
SDIR = os.path.join(GOLDEN, "reference", "secret")
ADIR = os.path.join(GOLDEN, "reference", "analyzer")


@pytest.fixture
def in_dir(request):
    old = os.getcwd()
    yield lambda d: os.chdir(d)
    os.chdir(old)


@pytest.mark.parametrize("case", CASES["scanner_cases"], ids=lambda c: c["name"])
def test_scanner_case(case, in_dir):
    in_dir(SDIR)
    content = open(case["input"], "rb").read()
    s = O.NewScanner(O.ParseConfig(case["config"]))
    got = s.Scan(case["input"], content)
    assert canon_secret(got) == case["want"]


@pytest.mark.parametrize("case", CASES["analyzer_cases"], ids=lambda c: c["name"])
def test_analyzer_case(case, in_dir):
    in_dir(ADIR)
    a = O.SecretAnalyzer(case["config"])
    content = open(case["input"], "rb").read()
    got = a.Analyze(case["input"], content, case["dir"])
    if case["want"] is None:
        assert got is None
    else:
        assert [canon_secret(x) for x in got["Secrets"]] == case["want"]["Secrets"]


@pytest.mark.parametrize("case", CASES["required_cases"], ids=lambda c: c["name"])
def test_required_case(case, in_dir):
    in_dir(ADIR)
    a = O.SecretAnalyzer("")
    assert a.Required(case["input"], os.path.getsize(case["input"])) == case["want"]


def test_integration_golden():
    root = os.path.join(GOLDEN, "reference", "integration", "secrets")
    integ = CASES["integration"]
    cfg = os.path.join(root, integ["config"])
    a = O.SecretAnalyzer(cfg)
    secrets = []
    for name in sorted(os.listdir(root)):
        path = os.path.join(root, name)
        if not a.Required(name, os.path.getsize(path)):
            continue
        res = a.Analyze(name, open(path, "rb").read(), root)
        if res:
            secrets.extend(res["Secrets"])
    O.sort_secrets(secrets)
    got = [{"Target": s["FilePath"], "Secrets": canon_secret(s)["Findings"]} for s in secrets]
    want = []
    for r in integ["results"]:
        fs = []
        for f in r["Secrets"]:
            g = {k: f[k] for k in ("RuleID", "Category", "Severity", "Title", "StartLine",
                                   "EndLine", "Match")}
            g["Code"] = {"Lines": [dict({"Highlighted": ""}, **ln) for ln in f["Code"]["Lines"]]}
            fs.append(g)
        want.append({"Target": r["Target"], "Secrets": fs})
    assert got == want
