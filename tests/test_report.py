"""End-to-end parity after the scan:

  * filesystem ingest (tsg_fs_pack, walker/fs.go + local/fs.go) of the integration
    fixture, then the JSON report of `trivy fs --security-checks vuln,secret
    --secret-config trivy-secret.yaml`, byte for byte against
    integration/testdata/secrets.json.golden (integration/fs_test.go:212-219)
  * layer stamping and cross-layer merging of secrets against the reference's own
    applier test case (pkg/fanal/applier/docker_test.go:332-480)

The golden file was written by a later trivy than this reference revision: its findings
carry `"Deleted": false`, a field pkg/fanal/types/secret.go does not have at this
revision.  The comparison drops exactly those lines from the golden, nothing else.
"""
import json
import os
import shutil

import pytest

from tests.conftest import GOLDEN
from trivy_amd import analyzer as A
from trivy_amd import report as R
from trivy_amd import walker as W

IDIR = os.path.join(GOLDEN, "reference", "integration")


def _golden_without_deleted():
    lines = open(os.path.join(IDIR, "secrets.json.golden")).read().split("\n")
    return "\n".join(l for l in lines if l.strip() != '"Deleted": false,')


@pytest.fixture
def fs_fixture(tmp_path):
    """integration/testdata/fixtures/fs/secrets laid out as the integration test sees it."""
    root = tmp_path / "testdata" / "fixtures" / "fs" / "secrets"
    root.mkdir(parents=True)
    for f in ("deploy.sh", "trivy-secret.yaml"):
        shutil.copy(os.path.join(IDIR, "secrets", f), root / f)
    old = os.getcwd()
    os.chdir(tmp_path)
    yield "testdata/fixtures/fs/secrets"
    os.chdir(old)


@pytest.mark.parametrize("mode", ["cpu", "emulated"])
def test_fs_json_report_matches_golden(fs_fixture, mode):
    an = A.SecretAnalyzer()
    an.Init(fs_fixture + "/trivy-secret.yaml")
    secrets = W.analyze_fs(an, fs_fixture, emulate_chunk=64 if mode == "emulated" else 0)
    rep = R.fs_report(fs_fixture, R.secrets_to_results(R.apply_layers([{"Secrets": secrets}])))
    assert R.write_json(rep) == _golden_without_deleted()


def test_fs_walk_gates(tmp_path):
    """walker/fs.go + Required + IsBinary: skipped dirs (.git, node_modules, --skip-dirs),
    --skip-files, lockfiles, extensions, binary and tiny files; relative paths, path order."""
    from trivy_amd import secret as S
    root = tmp_path / "tree"
    tok = b"export GITHUB_TOKEN=ghp_" + b"aB3dE5fG7hI9jK1lM3nO5pQ7rS9tU1vW3xY5" + b"\n"
    files = {"a/app.env": tok, "a/.git/config": tok, "node_modules/x/i.js": tok,
             "b/skip/me.txt": tok, "b/keep.txt": tok, "c/skipfile.txt": tok, "go.sum": tok,
             "img.png": tok, "bin.dat": b"\x00\x01" + tok, "tiny": b"ghp_", "z/README.md": tok}
    for p, c in files.items():
        (root / p).parent.mkdir(parents=True, exist_ok=True)
        (root / p).write_bytes(c)
    os.symlink(str(root / "b" / "keep.txt"), str(root / "b" / "link.txt"))
    fs = W.NativeFS(S.NewScanner(None), str(root), skip_files=[str(root / "c/skipfile.txt")],
                    skip_dirs=[str(root / "b/skip")])
    b = fs.batch
    assert [b.path(i) for i in range(b.nfiles)] == ["a/app.env", "b/keep.txt"]
    # walked: regular files outside skipped dirs and skip-files (incl. the ones Required drops)
    assert fs.walked == 8  # node_modules is dropped by Required, not by the walker


def test_apply_layers_reference_case():
    """docker_test.go:332-480 'happy path with removed and updated secret'."""
    def finding(rule, cat, title, line, match):
        return {"RuleID": rule, "Category": cat, "Severity": "CRITICAL", "Title": title,
                "StartLine": line, "EndLine": line, "Match": match,
                "Code": {"Lines": [{"Number": 1, "Content": match, "IsCause": True,
                                    "Annotation": "", "Truncated": False, "Highlighted": match,
                                    "FirstCause": True, "LastCause": True}]}}
    aws1 = finding("aws-access-key-id", "AWS", "AWS Access Key ID", 1,
                   "AWS_ACCESS_KEY_ID=********************")
    aws2 = finding("aws-access-key-id", "AWS", "AWS Access Key ID", 2,
                   "AWS_ACCESS_KEY_ID=********************")
    ghp = finding("github-pat", "GitHub", "GitHub Personal Access Token", 1,
                  "GITHUB_PAT=****************************************")
    d1 = "sha256:932da51564135c98a49a34a193d6cd363d8fa4184d957fde16c9d8527b3f3b02"
    i1 = "sha256:a187dde48cd289ac374ad8539930628314bc581a481cdb41409c9289419ddb72"
    d2 = "sha256:24df0d4e20c0f42d3703bf1f1db2bdd77346c7956f74f423603d651e8e5ae8a7"
    i2 = "sha256:aad63a9339440e7c3e1fff2b988991b9bfb81280042fa7f39a5e327023056819"
    layers = [
        {"Digest": d1, "DiffID": i1, "CreatedBy": "Line_1",
         "Secrets": [{"FilePath": "usr/secret.txt", "Findings": [aws1]}]},
        {"Digest": d2, "DiffID": i2, "CreatedBy": "Line_2",
         "Secrets": [{"FilePath": "usr/secret.txt", "Findings": [ghp, aws2]}]},
        {"Digest": d1, "DiffID": i1, "CreatedBy": "Line_3", "WhiteoutFiles": ["usr/secret.txt"]},
    ]
    got = R.apply_layers(layers)
    lay2 = {"Digest": d2, "DiffID": i2, "CreatedBy": "Line_2"}
    want = [{"FilePath": "usr/secret.txt",
             "Findings": [dict(ghp, Layer=lay2), dict(aws2, Layer=lay2)]}]
    assert got == want


def test_apply_layers_keeps_lower_layer_rules():
    """mergeSecrets: a lower layer's finding survives when the upper layer's version of
    the file has no finding with its RuleID; the upper layer wins per RuleID."""
    f = lambda rule, line: {"RuleID": rule, "StartLine": line, "Code": {"Lines": None}}
    got = R.apply_layers([
        {"Digest": "a", "Secrets": [{"FilePath": "x", "Findings": [f("r1", 1), f("r2", 2)]}]},
        {"Digest": "b", "Secrets": [{"FilePath": "x", "Findings": [f("r2", 9)]},
                                    {"FilePath": "w", "Findings": [f("r3", 3)]}]},
    ])
    assert [s["FilePath"] for s in got] == ["w", "x"]
    x = got[1]["Findings"]
    assert [(g["RuleID"], g["StartLine"], g["Layer"]["Digest"]) for g in x] == [
        ("r2", 9, "b"), ("r1", 1, "a")]


def test_apply_layers_duplicate_lower_rule_ids():
    """secretFindingsContains looks at the growing newSecret.Findings
    (applier/docker.go:280-284): of a lower layer's findings [r1@1, r1@5] the upper layer
    [r2@9] keeps only r1@1."""
    f = lambda rule, line: {"RuleID": rule, "StartLine": line, "Code": {"Lines": None}}
    got = R.apply_layers([
        {"Digest": "a", "Secrets": [{"FilePath": "x", "Findings": [f("r1", 1), f("r1", 5)]}]},
        {"Digest": "b", "Secrets": [{"FilePath": "x", "Findings": [f("r2", 9)]}]},
    ])
    assert [(g["RuleID"], g["StartLine"]) for g in got[0]["Findings"]] == [("r2", 9), ("r1", 1)]


def test_go_json_string_rules():
    assert R._go_string(b"<a & b>") == '"\\u003ca \\u0026 b\\u003e"'
    assert R._go_string(b"bad \xff byte") == '"bad � byte"'
    assert R._go_string("tab\tnl\ncr\r\x01") == '"tab\\tnl\\ncr\\r\\u0001"'
    assert R._go_string(" ") == '"\\u2028"'
    assert json.loads(R.write_json({"a": [1, None, {"b": True}], "c": {}, "d": []})) == \
        {"a": [1, None, {"b": True}], "c": {}, "d": []}


def test_source_tree_config0(tmp_path):
    """configs[0] at 6 MiB: the seeded source tree through the native fs ingest, scanned with
    the kernels' algorithm (emulated) == the exact CPU path, a file sample == the oracle; the
    .git dir, node_modules, lockfiles and the <10-byte file never reach Scan."""
    from oracle import secret as O
    from tests.helpers import canon_secret
    from trivy_amd import configs
    root = str(tmp_path / "tree")
    info = configs.source_tree(root, 6 << 20, seed=0)
    an = A.SecretAnalyzer()
    an.Init("")
    fs = W.NativeFS(an.scanner, root)
    paths = [fs.batch.path(i) for i in range(fs.batch.nfiles)]
    # the builtin global allow paths (tests, examples, vendor, docs, ...) drop more files
    assert 0 < fs.batch.nfiles < info["files"] - 5 and paths == sorted(paths)
    assert not any(p.startswith((".git/", "node_modules/")) or p in ("package-lock.json", "go.sum",
                                                                      "src/tiny.txt") for p in paths)
    emu = an.scanner.ScanBatch(fs.batch, emulate_chunk=256)
    assert emu == an.scanner.ScanBatch(fs.batch, nthreads=8)
    osc = O.NewScanner(None)
    for i in range(0, fs.batch.nfiles, 29):
        c = bytes(fs.batch.data[int(fs.batch.offsets[i]):int(fs.batch.offsets[i + 1])])
        assert canon_secret(emu[i]) == canon_secret(osc.Scan(paths[i], c)), paths[i]
    rules = {f["RuleID"] for r in emu if r["Findings"] for f in r["Findings"]}
    assert {"aws-access-key-id", "github-pat", "slack-access-token"} <= rules
