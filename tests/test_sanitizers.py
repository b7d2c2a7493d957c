"""ThreadSanitizer and AddressSanitizer builds of the host C++ (CPU only), running the
concurrency stress of the C ABI (tests/native/stress.cpp: tsg_scan_batch, ticketed
upload/submit/collect, tsg_queue and tsg_multi from 16 threads on emulated contexts, every
result byte-identical to the exact CPU path).  The round-2 verdict reproduced a batch
handed to the wrong caller; ASan found the Batch <-> queue-callback reference cycle of the
first ticketed version."""
import os
import sys

import pytest

from tests.conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.parametrize("kind", ["thread", "address"])
def test_stress_under_sanitizer(kind, tmp_path):
    import sanitize
    rc, log = sanitize.run(kind, str(tmp_path), nbytes=2 << 20)
    assert rc == 0 and log.rstrip().endswith("OK"), log[-4000:]
    assert "WARNING: ThreadSanitizer" not in log and "ERROR: AddressSanitizer" not in log
