"""bench.py's N>1 branch (BASELINE configs[2] / SURVEY §8e) executed on the leased GPU at world 2.

Two torchrun ranks share GPU 0 (``--device-map 0,0``; RCCL refuses two ranks on one device, so the group is gloo
and the waveform all-gather goes through the host — the code path is otherwise bench.py's own: env
rendezvous, per-rank device, barrier + synchronize around the timed steps, max-over-ranks timing, contiguous
prompt shards, all_gather_rows).  The gathered (2 x 32, 159744) waveforms must be bit-identical to one process
generating the same 64 prompt ids (per-prompt seeds make every clip shard-invariant; 32 prompts per rank keeps
every layer on the same kernel variant as the 64-prompt batch).  Reference sharding:
ldm/data/joinaudiodataset_anylen.py:165.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

ARGS = ["--steps", "1", "--warmup", "0", "--also-other-mode", "0", "--cpu-baseline", "0", "--extra-configs", "0",
        "--components", "0"]


def _run(cmd, tmp_path, name):
    # ALCM_KSPLIT=0: the K split is chosen by how full a layer's grid is, so 64 prompts in one process and 32 per rank
    # would sum the DiT FFN down-projection in different orders (same parity, DESIGN.md §2 "Sensitivity"); with it off
    # both batch sizes run the same kernel variants and the gathered waveforms must match bit for bit
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=REPO, ALCM_KSPLIT="0")
    with open(tmp_path / f"{name}.log", "w") as log:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=log, text=True, timeout=420, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + open(tmp_path / f"{name}.log").read()[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.fixture(scope="module")
def world1_64(tmp_path_factory):
    """One process generating the 64 prompt ids (the reference for both world-2 forms below)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    tmp = tmp_path_factory.mktemp("w1")
    one = _run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--batch", "64", "--dump-wav",
                str(tmp / "w1.npy")] + ARGS, tmp, "world1")
    assert one["config"]["global_batch"] == 64 and one["n_gpus"] == 1
    w1 = np.load(tmp / "w1.npy")
    assert w1.shape == (64, 159744) and np.isfinite(w1).all() and np.abs(w1).max() > 0
    return w1


def test_bench_world2_gathers_bit_identical_waveforms(tmp_path, world1_64):
    bench = os.path.join(REPO, "bench.py")
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr=127.0.0.1", "--master-port=29583", bench, "--gpus", "2", "--batch", "32",
                "--dist-backend", "gloo", "--device-map", "0,0", "--dump-wav", str(tmp_path / "w2.npy")] + ARGS,
               tmp_path, "world2")
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 64
    assert two["value"] > 0 and two["ms_per_step"] > 0
    w2 = np.load(tmp_path / "w2.npy")
    assert w2.shape == (64, 159744)
    assert np.array_equal(world1_64, w2)


def test_bench_spawns_ranks_itself(tmp_path, world1_64):
    """`bench.py --gpus 2` WITHOUT torch.distributed.run (the driver's N = 1 command form with N = 2): the parent
    starts the two ranks itself (bench.spawn_ranks) and relays rank 0's line; n_gpus is the process group's size."""
    two = _run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--batch", "32", "--dist-backend",
                "gloo", "--device-map", "0,0", "--dump-wav", str(tmp_path / "ws.npy")] + ARGS, tmp_path, "spawn")
    log = open(tmp_path / "spawn.log").read()
    assert "starting 2 ranks" in log
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 64 and two["value"] > 0
    assert np.array_equal(world1_64, np.load(tmp_path / "ws.npy"))


def test_bench_rccl_world1_collectives(tmp_path):
    """The RCCL lines of the N>1 path on the one leased GPU: torchrun world 1 with --force-collective runs
    init_process_group("nccl", device_id), barrier(device_ids), the device all_reduce of the step time and the
    device all_gather_into_tensor of the waveforms (distributed.py) — the code the driver's 8-GPU job runs — and the
    gathered waveforms must be bit-identical to the plain one-process run."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    bench = os.path.join(REPO, "bench.py")
    one = _run([sys.executable, bench, "--gpus", "1", "--batch", "32", "--dump-wav", str(tmp_path / "w1.npy")]
               + ARGS, tmp_path, "plain")
    rc = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", "--master-port=29587", bench, "--gpus", "1", "--batch", "32",
               "--dist-backend", "nccl", "--force-collective", "1", "--dump-wav", str(tmp_path / "wr.npy")] + ARGS,
              tmp_path, "rccl")
    log = open(tmp_path / "rccl.log").read()
    assert rc["n_gpus"] == 1 and rc["value"] > 0 and one["config"]["global_batch"] == 32
    assert rc["config"]["dist_backend"] == "nccl" and one["config"]["dist_backend"] is None
    w1, wr = np.load(tmp_path / "w1.npy"), np.load(tmp_path / "wr.npy")
    assert w1.shape == wr.shape == (32, 159744)
    assert np.array_equal(w1, wr), log[-3000:]
