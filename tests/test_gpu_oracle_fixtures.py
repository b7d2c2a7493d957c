"""The device path against the independent oracle at size, through committed fixtures
(SURVEY.md §8c): tools/gen_oracle_fixtures.py ran oracle/secret.py (a restatement of
scanner.go that shares no code with the product's resolver) over seeded corpora of
BASELINE configs[1] (16 MiB), configs[3] (2 MiB, 1,000 user rules) and configs[4]
(4 MiB, allow rules, exclude blocks, binary blobs) and stored every file's canonical
types.Secret.  Here the corpora are regenerated from the seeds (their sha256 must match),
scanned on the GPU (HIP kernels + host resolution) and compared file by file."""
import gzip
import json
import os

import pytest

from tests.conftest import GOLDEN
from tests.helpers import canon_secret
from tools.gen_oracle_fixtures import WORKLOADS, digest, workload
from trivy_amd import secret as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(WORKLOADS))
def test_device_equals_oracle_fixture(name):
    with gzip.open(os.path.join(GOLDEN, "oracle_bulk", name + ".json.gz"), "rt", encoding="utf-8") as f:
        rec = json.load(f)
    doc, args = workload(name)
    assert (rec["rules"], rec["MiB"], rec["seed"]) == WORKLOADS[name]
    assert digest(args) == rec["sha256"], "the regenerated corpus differs from the fixture's"
    sc = S.NewScanner(S.config_from_dict(doc)) if doc else S.NewScanner(None)
    got = sc.ScanBatch(args, device=0)
    bad = [a.FilePath for a, g, w in zip(args, got, rec["secrets"]) if canon_secret(g) != w]
    assert not bad, "%d of %d files differ from the oracle, e.g. %s" % (len(bad), len(args), bad[:5])
    assert sum(len(w["Findings"] or []) for w in rec["secrets"] if w) == rec["findings"] > 0
