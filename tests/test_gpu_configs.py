"""configs[3] / configs[4] parity on the device (see test_configs.py): HIP kernels +
host resolution == the exact CPU path, through the C ABI."""
import pytest

from trivy_amd import analyzer as A
from trivy_amd import configs
from trivy_amd import secret as S

pytestmark = pytest.mark.gpu


def test_user_rules_gpu_vs_exact():
    doc = configs.user_rules_doc(100, seed=4)
    sc = S.NewScanner(S.config_from_dict(doc))
    b = S.Batch.from_args(configs.mixed_batch(doc, 512 << 10, seed=61))
    want = sc.ScanBatch(b, nthreads=16)
    assert sc.ScanBatch(b, device=0) == want
    assert sum(len(x["Findings"] or []) for x in want) > 10


def test_allow_exclude_binary_gpu_vs_exact():
    doc = configs.allow_exclude_doc()
    sc = S.NewScanner(S.config_from_dict(doc))
    args = configs.mixed_batch(doc, 512 << 10, seed=62, plants_per_file=0.5, binary_frac=0.3)
    args = [a for a in args if not A.IsBinary(a.Content, len(a.Content))]
    b = S.Batch.from_args(args)
    want = sc.ScanBatch(b, nthreads=16)
    assert sc.ScanBatch(b, device=0) == want
    assert sum(len(x["Findings"] or []) for x in want) > 5
