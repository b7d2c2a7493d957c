"""Ingest straight into pinned slots (tsg_layer_pack_slot / tsg_fs_pack_slot /
tsg_layer_range_pack_slot).

The slot forms must pack exactly the batch of the pageable forms (tsg_layer_pack,
tsg_fs_pack, tsg_layer_range_pack: same bytes, offsets and paths; those are pinned by
test_walker.py / test_report.py against the walker semantics of pkg/fanal/walker/tar.go and
fs.go), and scanning the slot must give the results of scanning that batch.  CPU tests run
on an emulated context (TSG_CTX_EMULATE: the kernels' algorithm on the CPU over the same
slots); test_gpu.py runs the same flow on the device."""
import os

import numpy as np
import pytest

from tests.conftest import ROOT
from tests.test_walker import layer_bytes
from trivy_amd import analyzer as A
from trivy_amd import configs
from trivy_amd import secret as S
from trivy_amd import walker as W


@pytest.fixture(scope="module")
def scanner():
    return S.NewScanner(None)


def _same_batch(a, b):
    assert a.nfiles == b.nfiles
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.path_offsets, b.path_offsets)
    n = int(a.offsets[-1])
    assert bytes(a.data[:n]) == bytes(b.data[:n])
    assert [a.path(i) for i in range(a.nfiles)] == [b.path(i) for i in range(b.nfiles)]


def test_layer_pack_slot_matches_pack(scanner):
    tar = layer_bytes()
    ctx = S.GpuContext(scanner, 0, emulate=True)
    ref = W.NativeLayer(scanner, tar, skip_files=["app/skipme.txt"])
    got = W.SlotIngest.layer(ctx, tar, skip_files=["app/skipme.txt"])
    _same_batch(got.batch, ref.batch)
    assert (got.opq, got.wh, got.walked) == (ref.opq, ref.wh, ref.walked)
    assert got.scan() == scanner.ScanBatch(ref.batch)
    got.release()
    ctx.close()


def test_layer_pack_slot_seeded(scanner):
    tar = configs.layer_tar(3 << 20, seed=7, binary_frac=0.1)
    ctx = S.GpuContext(scanner, 0, emulate=True)
    ref = W.NativeLayer(scanner, tar)
    got = W.SlotIngest.layer(ctx, tar)
    _same_batch(got.batch, ref.batch)
    assert got.scan() == scanner.ScanBatch(ref.batch)
    # the slot is reused after release: a second pack into the same context
    got.release()
    again = W.SlotIngest.layer(ctx, tar)
    _same_batch(again.batch, ref.batch)
    again.release()
    ctx.close()


@pytest.mark.parametrize("world", [1, 3])
def test_layer_range_pack_slot_matches_range_pack(scanner, world):
    tar = configs.layer_tar(2 << 20, seed=9)
    ctx = S.GpuContext(scanner, 0, emulate=True)
    refs = W.pack_layer_ranges(scanner, tar, world)
    rngs = [W.LayerRange(tar, r, world) for r in range(world)]
    infos = [g.info for g in rngs]
    confirmed = {}
    while True:
        st = W.layer_chain_step(infos, confirmed)
        if st[0] == "done":
            break
        confirmed[st[1]] = rngs[st[1]].sync(st[2])
    for g, pos in zip(rngs, st[1]):
        g.sync(pos)
    prior = []
    for r, g in enumerate(rngs):
        got = W.SlotIngest.layer_range(ctx, g, prior_dirs=prior)
        _same_batch(got.batch, refs[r].batch)
        assert got.scan() == scanner.ScanBatch(refs[r].batch)
        got.release()
        prior = prior + g.dirs()
    ctx.close()


def _tree(root):
    """A tree with small, large (> 64 KiB, read straight into the slot), binary, skipped,
    tiny (Required) and nested files."""
    os.makedirs(os.path.join(root, "a/b/c"))
    os.makedirs(os.path.join(root, "node_modules/m"))
    os.makedirs(os.path.join(root, ".git"))
    os.makedirs(os.path.join(root, "skipdir"))
    tok = "ghp_" + "aB3dE5fG7hI9jK1lM3nO5pQ7rS9tU1vW3xY5"
    files = {
        "a/small.txt": "export GITHUB_TOKEN=%s\n" % tok,
        "a/b/large.txt": ("filler line of text\n" * 5000) + "token: %s\n" % tok + "tail\n" * 100,
        "a/b/c/deep.env": "x=1\nGITHUB_TOKEN=%s\n" % tok,
        "a/bin_small.dat": "\x00\x01binary %s" % tok,
        "a/bin_large.dat": "\x00" + "y" * 100000 + tok,
        "a/tiny": "ghp_x",
        "node_modules/m/index.js": "GITHUB_TOKEN=%s\n" % tok,
        ".git/config": "GITHUB_TOKEN=%s\n" % tok,
        "skipdir/s.txt": "GITHUB_TOKEN=%s\n" % tok,
        "a/skipme.txt": "GITHUB_TOKEN=%s\n" % tok,
        "top.txt": "nothing here\n" * 10,
        "a/empty.txt": "",
    }
    for p, c in files.items():
        with open(os.path.join(root, p), "w", encoding="latin-1") as f:
            f.write(c)
    return files


def test_fs_pack_gates(tmp_path, scanner):
    root = str(tmp_path / "t")
    _tree(root)
    fs = W.NativeFS(scanner, root, skip_files=[os.path.join(root, "a/skipme.txt")],
                    skip_dirs=[os.path.join(root, "skipdir")])
    paths = [fs.batch.path(i) for i in range(fs.batch.nfiles)]
    # path order; binary files, Required's skip dirs / size, .git and skip lists left out
    assert paths == ["a/b/c/deep.env", "a/b/large.txt", "a/small.txt", "top.txt"]
    assert fs.walked == 9  # regular files outside the skip lists and skipped dirs (incl. gated ones)
    big = open(os.path.join(root, "a/b/large.txt"), "rb").read()
    k = paths.index("a/b/large.txt")
    assert bytes(fs.batch.data[int(fs.batch.offsets[k]):int(fs.batch.offsets[k + 1])]) == big


def test_fs_pack_slot_matches_pack(tmp_path, scanner):
    root = str(tmp_path / "t")
    _tree(root)
    configs.source_tree(os.path.join(root, "src"), 3 << 20, seed=1)
    ctx = S.GpuContext(scanner, 0, emulate=True)
    ref = W.NativeFS(scanner, root)
    got = W.SlotIngest.fs(ctx, root)
    _same_batch(got.batch, ref.batch)
    assert got.walked == ref.walked
    res = got.scan()
    assert res == scanner.ScanBatch(ref.batch)
    assert sum(len(r["Findings"] or []) for r in res) > 0
    got.release()
    ctx.close()


def test_fs_pack_slot_analyzer_equivalence(tmp_path):
    """analyze_fs over the slot form equals the exact CPU path over the same tree."""
    root = str(tmp_path / "t")
    _tree(root)
    an = A.SecretAnalyzer(S.NewScanner(None), "")
    ctx = S.GpuContext(an.scanner, 0, emulate=True)
    got = W.SlotIngest.fs(ctx, root, config_path=an.configPath)
    res = A.sort_secrets([r for r in got.scan() if r["Findings"]])
    assert res == W.analyze_fs(an, root)
    got.release()
    ctx.close()


def test_slot_ingest_errors(scanner, tmp_path):
    ctx = S.GpuContext(scanner, 0, emulate=True)
    with pytest.raises(Exception):
        W.SlotIngest.fs(ctx, str(tmp_path / "missing"))
    with pytest.raises(Exception):
        W.SlotIngest.layer(ctx, b"\x01" * 1024)  # not a tar: failed to extract the archive
    # a failed pack holds no slot: the context still serves a full batch
    ok = W.SlotIngest.layer(ctx, layer_bytes())
    assert ok.batch.nfiles > 0
    ok.release()
    ctx.close()


@pytest.mark.parametrize("slot_mib", [1, 256])
def test_layer_scan_pipelined_matches_pack(scanner, slot_mib):
    """tsg_layer_scan (pieces of slot_mib, overlapped) == scanning tsg_layer_pack's batch:
    the same files, paths, order, results, opq / wh / walked."""
    tar = configs.layer_tar(6 << 20, seed=11, binary_frac=0.1)
    ctx = S.GpuContext(scanner, 0, emulate=True, slot_mib=slot_mib)
    ref = W.NativeLayer(scanner, tar)
    paths, res, opq, wh, walked = W.scan_layer_pipelined(ctx, tar)
    assert paths == [ref.batch.path(i) for i in range(ref.batch.nfiles)]
    assert res == scanner.ScanBatch(ref.batch)
    assert (opq, wh, walked) == (ref.opq, ref.wh, ref.walked)
    assert sum(len(r["Findings"] or []) for r in res) > 10
    ctx.close()


@pytest.mark.parametrize("slot_mib", [1, 256])
def test_fs_scan_pipelined_matches_pack(tmp_path, scanner, slot_mib):
    root = str(tmp_path / "t")
    _tree(root)
    configs.source_tree(os.path.join(root, "src"), 4 << 20, seed=2)
    ctx = S.GpuContext(scanner, 0, emulate=True, slot_mib=slot_mib)
    ref = W.NativeFS(scanner, root)
    paths, res, _, _, walked = W.scan_fs_pipelined(ctx, root)
    assert paths == [ref.batch.path(i) for i in range(ref.batch.nfiles)]
    assert res == scanner.ScanBatch(ref.batch)
    assert walked == ref.walked
    ctx.close()


def test_pipelined_scan_errors_leave_no_pending(scanner, tmp_path):
    ctx = S.GpuContext(scanner, 0, emulate=True, slot_mib=1)
    with pytest.raises(Exception):
        W.scan_layer_pipelined(ctx, b"\x01" * 1024)
    with pytest.raises(Exception):
        W.scan_fs_pipelined(ctx, str(tmp_path / "missing"))
    assert ctx.pending() == 0
    paths, res, _, _, _ = W.scan_layer_pipelined(ctx, layer_bytes())
    assert len(paths) == len(res) > 0
    ctx.close()


@pytest.mark.parametrize("world", [2, 3])
def test_fs_pack_shard_union_is_fs_pack(tmp_path, scanner, world):
    """tsg_fs_pack_shard: each rank reads only its contiguous byte run of the listed tree;
    the shards in rank order are tsg_fs_pack's batch (files, bytes, paths), walked is the
    whole tree's."""
    root = str(tmp_path / "t")
    _tree(root)
    configs.source_tree(os.path.join(root, "src"), 2 << 20, seed=3)
    ref = W.NativeFS(scanner, root)
    parts = [W.NativeFS(scanner, root, rank=r, world=world) for r in range(world)]
    paths = [p.batch.path(i) for p in parts for i in range(p.batch.nfiles)]
    assert paths == [ref.batch.path(i) for i in range(ref.batch.nfiles)]
    data = b"".join(bytes(p.batch.data[:int(p.batch.offsets[-1])]) for p in parts)
    assert data == bytes(ref.batch.data[:int(ref.batch.offsets[-1])])
    assert all(p.walked == ref.walked for p in parts)
    assert min(p.batch.nfiles for p in parts) > 0


@pytest.mark.parametrize("seed", [1, 2])
def test_fs_scan_drops_binary_across_pieces(tmp_path, scanner, seed):
    """tsg_fs_scan reads every listed file into its piece and drops the binary ones when the
    pieces are joined: with many binary files (some before, between and after text files,
    some at piece boundaries of 1 MiB slots) the joined result equals scanning tsg_fs_pack's
    batch, file for file."""
    rng = np.random.default_rng(seed)
    root = str(tmp_path / "t")
    os.makedirs(root)
    tok = "ghp_" + "aB3dE5fG7hI9jK1lM3nO5pQ7rS9tU1vW3xY5"
    for i in range(120):
        d = os.path.join(root, "d%d" % (i % 7))
        os.makedirs(d, exist_ok=True)
        n = int(rng.integers(10, 300_000))
        if rng.random() < 0.4:  # binary: a control byte in the first 300 bytes
            body = bytes(rng.integers(0, 256, n, dtype=np.uint8))
            body = body[:5] + b"\x01" + body[6:]
        else:
            body = (b"line of text %d\n" % i) * (n // 16) + ("GITHUB_TOKEN=%s\n" % tok).encode()
        with open(os.path.join(d, "f%03d.txt" % i), "wb") as f:
            f.write(body)
    ctx = S.GpuContext(scanner, 0, emulate=True, slot_mib=1)
    ref = W.NativeFS(scanner, root)
    paths, res, _, _, walked = W.scan_fs_pipelined(ctx, root)
    assert paths == [ref.batch.path(i) for i in range(ref.batch.nfiles)]
    assert res == scanner.ScanBatch(ref.batch)
    assert walked == ref.walked == 120
    assert 40 < len(paths) < 100
    ctx.close()


_EMFILE_CHILD = r"""
import os, sys, errno
sys.path.insert(0, sys.argv[2])
from trivy_amd import secret as S, walker as W, _native as N
sc = S.NewScanner(None)
held = []
try:  # take every descriptor but one: the walk's directory gets it, no file open can succeed
    while True:
        held.append(os.open("/dev/null", os.O_RDONLY))
except OSError as e:
    assert e.errno == errno.EMFILE
os.close(held.pop())
try:
    W.NativeFS(sc, sys.argv[1])
    print("PACKED")
except N.NativeError as e:
    print("ERROR", e)
"""


def test_fs_pack_open_error_fails_scan(tmp_path):
    """A file the walk listed but cannot open for a reason other than permissions (here a
    descriptor table that stays full past open_at_retry's wait) fails the scan like the
    reference's "unable to open" (analyzer.go:411-416) instead of silently dropping the file
    (ADVICE r4).  Run in a child process with a low descriptor limit."""
    import subprocess
    import sys
    root = tmp_path / "t"
    (root / "d").mkdir(parents=True)
    for i in range(3):
        (root / "d" / ("f%d.txt" % i)).write_text("token = %d\n" % i)
    prog = "import resource; resource.setrlimit(resource.RLIMIT_NOFILE, (64, 64))\n" + _EMFILE_CHILD
    r = subprocess.run([sys.executable, "-c", prog, str(root), ROOT], capture_output=True, text=True, timeout=120)
    assert "ERROR" in r.stdout and "unable to open" in r.stdout, r.stdout + r.stderr
