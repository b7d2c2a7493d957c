"""The oracle fixtures at size (tools/gen_oracle_fixtures.py, tests/golden/oracle_bulk/) on
the CPU: the seeds regenerate the stored corpora exactly (sha256), and the product's exact
CPU path (tsg_scan_cpu_batch) and the GPU algorithm emulated on the CPU both equal the
oracle on every file.  tests/test_gpu_oracle_fixtures.py runs the same comparison on the
device."""
import gzip
import json
import os

import pytest

from tests.conftest import GOLDEN
from tests.helpers import canon_secret
from tools.gen_oracle_fixtures import SAMPLES, WORKLOADS, digest, sample_expect, workload
from trivy_amd import secret as S


@pytest.mark.parametrize("name", sorted(WORKLOADS))
def test_exact_and_emulated_equal_oracle_fixture(name):
    with gzip.open(os.path.join(GOLDEN, "oracle_bulk", name + ".json.gz"), "rt", encoding="utf-8") as f:
        rec = json.load(f)
    doc, args = workload(name)
    assert digest(args) == rec["sha256"]
    sc = S.NewScanner(S.config_from_dict(doc)) if doc else S.NewScanner(None)
    for got in (sc.ScanBatch(args, nthreads=8), sc.ScanBatch(args, emulate_chunk=256, nthreads=8)):
        bad = [a.FilePath for a, g, w in zip(args, got, rec["secrets"]) if canon_secret(g) != w]
        assert not bad, bad[:5]


@pytest.mark.parametrize("name", sorted(SAMPLES))
def test_oracle_samples_regenerate_and_match_exact(name, tmp_path):
    """The per-test oracle samples the GPU tests and smoke() read (tests/golden/oracle_small/):
    their seeds regenerate the stored inputs (sha256, inside sample_expect), and the exact CPU
    path equals the stored oracle results on every file."""
    doc, args = SAMPLES[name](str(tmp_path))
    want = sample_expect(name, args)
    sc = S.NewScanner(S.config_from_dict(doc)) if doc else S.NewScanner(None)
    got = sc.ScanBatch(args, nthreads=8)
    bad = [a.FilePath for a, g, w in zip(args, got, want) if canon_secret(g) != w]
    assert len(got) == len(want) and not bad, bad[:5]
