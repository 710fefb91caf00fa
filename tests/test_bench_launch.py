"""bench.py --gpus N: the launcher's plumbing on CPU (no GPU is touched).

`launch_plan` decides, before any HIP call, whether this process is a rank or must start N ranks, and rejects the
mismatches (--gpus vs WORLD_SIZE under torch.distributed.run, a --device-map of the wrong length, more GPUs than are
visible); `spawn_ranks` starts the ranks through torch.distributed.run and relays rank 0's JSON line.  The GPU form
(bench.py --gpus 2 --device-map 0,0 without torchrun, bit-identical gathered waveforms) is
tests/test_gpu_dist.py::test_bench_spawns_ranks_itself.  Reference sharding: ldm/data/joinaudiodataset_anylen.py:164-165.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launch_plan_single_and_spawn():
    assert bench.launch_plan(1, None, {}, 1) is None              # N = 1: this process is the rank
    assert bench.launch_plan(8, None, {}, 8) == 8                 # N = 8 without torchrun: spawn 8
    assert bench.launch_plan(2, "0,0", {}, 1) == 2                # rehearsal: two ranks on GPU 0
    assert bench.launch_plan(8, None, {"WORLD_SIZE": "8"}, 0) is None  # started by torch.distributed.run


@pytest.mark.parametrize("gpus,dmap,env,vis,msg", [
    (8, None, {"WORLD_SIZE": "1"}, 8, "WORLD_SIZE=1"),
    (2, None, {"WORLD_SIZE": "2"}, 2, None),
    (8, None, {}, 1, "needs 8 GPUs, 1 visible"),
    (2, "0,1", {}, 1, "needs 2 GPUs, 1 visible"),
    (2, "0", {}, 2, "names 1 GPUs for --gpus 2"),
    (0, None, {}, 8, "at least one"),
    (1, None, {}, 0, "needs 1 GPUs, 0 visible"),
])
def test_launch_plan_mismatches(gpus, dmap, env, vis, msg):
    if msg is None:
        assert bench.launch_plan(gpus, dmap, env, vis) is None
        return
    with pytest.raises(ValueError, match=msg):
        bench.launch_plan(gpus, dmap, env, vis)


def test_visible_gpus_from_env():
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,1,2"}) == 3
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,1,2", "ROCR_VISIBLE_DEVICES": "4"}) == 1
    assert bench.visible_gpus({"CUDA_VISIBLE_DEVICES": ""}) == 0


def test_bench_refuses_more_gpus_than_visible():
    """On this CPU container no GPU is visible: --gpus 2 must fail fast with the message, before any rank starts."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "needs 2 GPUs, 1 visible" in r.stderr
    assert "starting" not in r.stderr and r.stdout == ""


def test_bench_refuses_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


RANK_SCRIPT = r'''
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
w = dist.get_world_size()
if dist.get_rank() == 0:
    print("not json, rank 0 chatter")
    print(json.dumps({"world": w, "argv": sys.argv[1:], "master": os.environ["MASTER_ADDR"]}), flush=True)
dist.barrier()
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == int(os.environ["RANK"]) and 3 or 0)
'''


def test_spawn_ranks_forwards_flags_and_relays_rank0(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc = bench.spawn_ranks(2, ["--gpus", "2", "--steps", "7", "--dist-backend", "gloo"], script=str(script))
    out, err = capfd.readouterr()
    assert rc == 0, err[-3000:]
    lines = [l for l in out.splitlines() if l.strip()]
    assert len(lines) == 1, out            # only rank 0's JSON line on stdout; other output goes to stderr
    d = json.loads(lines[0])
    assert d == {"world": 2, "argv": ["--gpus", "2", "--steps", "7", "--dist-backend", "gloo"], "master": "127.0.0.1"}
    assert "rank 0 chatter" in err


def test_spawn_ranks_propagates_failure(tmp_path, monkeypatch):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    monkeypatch.setenv("FAIL_RANK", "1")
    assert bench.spawn_ranks(2, [], script=str(script)) != 0
