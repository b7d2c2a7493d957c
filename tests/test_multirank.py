"""The N>1 path on the CPU: two ranks over gloo (127.0.0.1), each scanning an LPT share of
the files with the emulated kernel algorithm; rank 0's gathered results must equal a
single-process scan.  No collective touches the data path."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

from tests.conftest import ROOT
from trivy_amd.shard import lpt_shards


def test_lpt_shards_partition_and_balance():
    sizes = [5, 1, 9, 3, 3, 7, 2, 8, 0, 4]
    sh = lpt_shards(sizes, 3)
    assert sorted(i for s in sh for i in s) == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in s) for s in sh]
    assert max(loads) - min(loads) <= max(sizes)
    assert lpt_shards(sizes, 1) == [list(range(len(sizes)))]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, %(root)r)
    import torch.distributed as dist
    from tests.helpers import canon_secret
    from trivy_amd import corpus, secret as S
    from trivy_amd.shard import scan_sharded, findings_sorted
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d",
                            rank=int(sys.argv[1]), world_size=2)
    b, _ = corpus.make_corpus(1 << 20, seed=17, plants_per_mib=200)
    args = [S.ScanArgs(b.path(i), bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])]))
            for i in range(b.nfiles)]
    sc = S.NewScanner(None)
    res = scan_sharded(sc, args, dist.get_rank(), 2, dist=dist, emulate_chunk=64)
    if dist.get_rank() == 0:
        want = sc.ScanBatch(args)
        assert res == want
        n = len(findings_sorted(res))
        assert n > 10
        print("OK", n)
    dist.destroy_process_group()
""")


def test_two_ranks_gloo(tmp_path):
    port = _free_port()
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"root": ROOT, "port": port})
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, str(script), str(r)], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "OK" in outs[0]


LAYER_WORKER = textwrap.dedent("""
    import io, sys
    sys.path.insert(0, %(root)r)
    import torch.distributed as dist
    from tests.helpers import canon_secret
    from trivy_amd import analyzer as A, configs, secret as S, walker as W
    from trivy_amd.shard import scan_layer_sharded
    rank = int(sys.argv[1])
    device = %(device)r
    if rank == %(fail_rank)d:  # an ingest failure on this rank alone
        def bad(self, *a, **k):
            raise RuntimeError("injected failure")
        W.LayerRange.dirs = bad
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d",
                            rank=rank, world_size=2)
    tar = configs.layer_tar(%(nbytes)d, seed=21)
    an = A.SecretAnalyzer(S.NewScanner(None), "")
    try:
        out = scan_layer_sharded(an, tar, rank, 2, dist=dist, device=device,
                                 emulate_chunk=0 if device is not None else 64)
    except RuntimeError as e:
        print("RAISED", e)
        sys.exit(3)
    if rank == 0:
        got, opq, wh = out
        want, opq2, wh2 = W.analyze_layer(an, io.BytesIO(tar))
        assert [canon_secret(s) for s in got] == [canon_secret(s) for s in want]
        assert (opq, wh) == (opq2, wh2) and len(got) > 10
        if device is not None:  # the device union against the oracle's committed results
            from tools.gen_oracle_fixtures import sample_expect
            lay = W.NativeLayer(an.scanner, tar)
            b = lay.batch
            args = [S.ScanArgs(b.path(i), bytes(b.data[int(b.offsets[i]):int(b.offsets[i + 1])]))
                    for i in range(b.nfiles)]
            want = dict(zip([a.FilePath for a in args], sample_expect("two_rank_layer", args)))
            for s in got[::4]:
                assert canon_secret(s) == want[s["FilePath"]]
        print("OK", len(got))
    else:
        assert out is None
    dist.destroy_process_group()
""")


def _run_layer_ranks(tmp_path, device=None, fail_rank=-1, nbytes=1 << 20):
    port = _free_port()
    script = tmp_path / "wl.py"
    script.write_text(LAYER_WORKER % {"root": ROOT, "port": port, "device": device,
                                      "fail_rank": fail_rank, "nbytes": nbytes})
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, str(script), str(r)], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    try:
        outs = [p.communicate(timeout=240)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return procs, outs


def test_two_ranks_layer_gloo(tmp_path):
    """configs[2]: one layer's files sharded over 2 ranks == the single-process layer scan."""
    procs, outs = _run_layer_ranks(tmp_path)
    assert all(p.returncode == 0 for p in procs), outs
    assert "OK" in outs[0]


def test_two_ranks_layer_error_on_one_rank(tmp_path):
    """An ingest failure on one rank of the distributed index raises on every rank instead
    of leaving the others waiting in a collective."""
    procs, outs = _run_layer_ranks(tmp_path, fail_rank=1)
    assert [p.returncode for p in procs] == [3, 3], outs
    assert all("rank 1: injected failure" in o for o in outs), outs


@pytest.mark.gpu
def test_two_ranks_layer_gpu(tmp_path):
    """configs[2] on the device: the distributed index (index="range") at world size 2 over
    gloo, both ranks sharing the one GPU; rank 0's union == the single-process layer scan,
    and a sample of it == the oracle."""
    procs, outs = _run_layer_ranks(tmp_path, device=0, nbytes=6 << 20)
    assert all(p.returncode == 0 for p in procs), outs
    assert "OK" in outs[0]


FS_WORKER = textwrap.dedent("""
    import sys
    sys.path.insert(0, %(root)r)
    import torch.distributed as dist
    from tests.helpers import canon_secret
    from trivy_amd import analyzer as A, configs, secret as S, walker as W
    from trivy_amd.shard import scan_fs_sharded
    rank = int(sys.argv[1])
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d",
                            rank=rank, world_size=2)
    root = %(tree)r
    if rank == 0:
        configs.source_tree(root, 2 << 20, seed=23)
    dist.barrier()
    an = A.SecretAnalyzer(S.NewScanner(None), "")
    device = %(device)r
    out = scan_fs_sharded(an, root, rank, 2, dist=dist, device=device,
                          emulate_chunk=0 if device is not None else 64)
    if rank == 0:
        want = W.analyze_fs(an, root)
        assert [canon_secret(s) for s in out] == [canon_secret(s) for s in want]
        assert len(out) > 10
        print("OK", len(out))
    else:
        assert out is None
    dist.destroy_process_group()
""")


def _run_fs_ranks(tmp_path, device=None):
    port = _free_port()
    script = tmp_path / "wf.py"
    script.write_text(FS_WORKER % {"root": ROOT, "port": port, "tree": str(tmp_path / "tree"),
                                   "device": device})
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, str(script), str(r)], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    try:
        outs = [p.communicate(timeout=240)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return procs, outs


def test_two_ranks_fs_gloo(tmp_path):
    """configs[0] over 2 ranks: each reads only its byte run of the tree (tsg_fs_pack_shard);
    rank 0's gathered findings == the single-process fs analysis."""
    procs, outs = _run_fs_ranks(tmp_path)
    assert all(p.returncode == 0 for p in procs), outs
    assert "OK" in outs[0]


@pytest.mark.gpu
def test_two_ranks_fs_gpu(tmp_path):
    """The same with both ranks scanning on the one GPU (as bench.py --gpus N would on N)."""
    procs, outs = _run_fs_ranks(tmp_path, device=0)
    assert all(p.returncode == 0 for p in procs), outs
    assert "OK" in outs[0]
