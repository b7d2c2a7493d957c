"""bench.py's GPU-count contract on the CPU (emulated contexts: the kernels' algorithm on the
host over the same slots, lanes and tickets).

* --gpus N without torchrun drives N device contexts from one process (tsg_multi) and
  reports n_gpus = N;
* under torchrun each rank drives one device, and WORLD_SIZE must equal --gpus;
* asking for more GPUs than the process sees fails, never runs on fewer."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--gb", "0.01", "--batch-mib", "2", "--steps", "2", "--warmup", "1", "--cpu-mib", "2"]


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=timeout, env=e, cwd=ROOT)


def _line(r):
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_two_devices_one_process_emulated():
    line = _line(_run(["--gpus", "2", "--emulate"] + SMALL))
    assert line["n_gpus"] == 2
    assert line["config"]["devices"] == [0, 1]
    assert "tsg_multi" in line["config"]["parallelism"]
    per = line["kernels"]["per_device"]
    assert [p["device"] for p in per] == [0, 1] and all(p["batches"] > 0 for p in per)
    # both devices' shares were scanned in every step: the job is twice one GPU's bytes
    assert line["config"]["job_bytes"] == 2 * line["config"]["bytes_per_gpu"]
    assert line["checks"]["sample_device_eq_exact_cpu"] is True
    one = _line(_run(["--gpus", "1", "--emulate", "--no-cpu-baseline"] + SMALL))
    assert one["n_gpus"] == 1
    # device 0's share is the same corpus in both runs (seeded by the GPU index)
    assert one["config"]["bytes_per_gpu"] == line["config"]["bytes_per_gpu"]


def test_more_gpus_than_visible_fails():
    r = _run(["--gpus", "2"] + SMALL, env={"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert "refusing to run on fewer" in r.stderr


def test_world_size_must_equal_gpus():
    r = _run(["--gpus", "3", "--emulate"] + SMALL, env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_torchrun_two_ranks_emulated():
    """The driver's N>1 form: torchrun, one rank per (emulated) device, gloo timing."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29631", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--emulate", "--no-cpu-baseline"] + SMALL
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert "torchrun" in line["config"]["parallelism"]
    assert line["config"]["job_bytes"] == 2 * line["config"]["bytes_per_gpu"]


def test_e2e_fs_configs4_mix_emulated():
    """configs[4]'s mix in the timed end-to-end path: 30 % of the tree's bytes binary blobs,
    half of them with a text head that IsBinary (utils.go:71-89) passes to Scan, under the
    allow-rule / exclude-block rule set loaded from a trivy-secret.yaml; the first step's
    results must equal the exact CPU path's (the bench checks it and fails otherwise)."""
    r = _run(["--e2e", "fs", "--e2e-mib", "8", "--rules", "allow-exclude", "--binary-frac", "0.3",
              "--binary-text-head", "0.5", "--emulate", "--steps", "1", "--warmup", "1"])
    line = _line(r)
    assert line["checks"]["step1_eq_exact_cpu"] is True
    assert line["config"]["rule_set"] == "allow-exclude" and line["config"]["binary_frac"] == 0.3
    assert "with a text head" in line["data"] and line["config"]["findings"] > 0
    # the dropped half is read (input bytes) but not scanned
    assert line["config"]["scanned_bytes"] < 0.9 * line["config"]["input_bytes"]


def test_eight_devices_one_process_emulated():
    """N = 8 in one process, as a single trivy process binds a node (tsg_multi over 8
    emulated devices; image.go:210-234's per-layer goroutines and gather): every device gets
    its share, its own slots and lanes at the run's depth, and the resolver pool sized for
    eight devices; the sample check and the per-step findings check pass."""
    line = _line(_run(["--gpus", "8", "--emulate", "--gb", "0.004", "--batch-mib", "1", "--steps", "2",
                       "--warmup", "1", "--depth", "4", "--cpu-mib", "1"], timeout=600))
    assert line["n_gpus"] == 8
    assert line["config"]["devices"] == list(range(8))
    per = line["kernels"]["per_device"]
    assert [p["device"] for p in per] == list(range(8)) and all(p["batches"] > 0 for p in per)
    assert line["config"]["job_bytes"] == 8 * line["config"]["bytes_per_gpu"]
    assert line["roofline"]["aggregate"]["gpus"] == 8
    assert line["checks"]["sample_device_eq_exact_cpu"] is True


def test_torchrun_eight_ranks_emulated():
    """The driver's N = 8 form on the CPU: torchrun, eight ranks over gloo, one emulated
    device each; barrier + max-over-ranks timing, rank 0's line alone."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", "29641", os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--emulate", "--no-cpu-baseline", "--gb", "0.004", "--batch-mib", "1",
           "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and "torchrun" in line["config"]["parallelism"]
    assert line["config"]["job_bytes"] == 8 * line["config"]["bytes_per_gpu"]
    assert line["roofline"]["aggregate"]["gpus"] == 8


def test_rehearsal_line_claims_no_more_gpus_than_used():
    """--rehearse-shared-gpu (ranks sharing GPUs): the line reports the distinct GPUs it used
    and no throughput value or aggregate roofline, so it cannot read as a multi-GPU run."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29651", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--emulate", "--rehearse-shared-gpu", "--no-cpu-baseline"] + SMALL
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["n_gpus"] == 1 and line["value"] is None
    assert line["rehearsal"]["ranks"] == 2 and line["roofline"]["aggregate"] is None
