"""Multi-GPU prompt sharding: one process per GPU, RCCL all-gather of waveforms over xGMI.

The path shards embarrassingly: prompts are independent and the
per-prompt seeds make every clip independent of the shard it lands on.  Each rank
generates a contiguous shard of the global batch; the only collective is one
``all_gather_into_tensor`` of the decoded waveforms (backend "nccl" == RCCL on ROCm,
"gloo" for the CPU tests).  Replaces the reference's rank-strided batch split
(ldm/data/joinaudiodataset_anylen.py:165) used for its multi-GPU work.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of n items for `rank` (sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def init_from_env(backend: Optional[str] = None, device: Optional[int] = None,
                  force: bool = False) -> Tuple[int, int, int]:
    """torch.distributed init from RANK/WORLD_SIZE/LOCAL_RANK (torchrun); returns (rank, world, local).

    ``device``: the GPU this rank drives.  It is made current BEFORE the process group exists and, for
    nccl (RCCL), bound to the group (``device_id``), so collectives and barriers never guess a device.
    ``force``: create the group even at world 1 (the one-GPU rehearsal of the N>1 code path: every collective
    below then really runs, over RCCL with backend nccl)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device is not None:
        torch.cuda.set_device(device)
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = torch.device("cuda", device)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def barrier(group=None) -> None:
    """dist.barrier on the rank's own device for nccl (no device guess), plain for gloo."""
    if dist.get_backend(group) == "nccl":
        dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=group)


def all_reduce_max(value: float, group=None) -> float:
    """Max of a host scalar over ranks (bench timing): on the device for nccl, on the host for gloo."""
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def all_gather_rows_async(local: torch.Tensor, n_total: int, group=None):
    """all_gather_rows without waiting: -> (out, work).  Over RCCL (equal shards, device tensors) the gather is
    enqueued on the collective's own stream behind the producer of ``local`` and ``work.wait()`` orders the caller's
    current stream after it, so the next batch's kernels overlap the waveform exchange (bench.py keeps one gather in
    flight).  Other cases (gloo, ragged shards, no process group) complete before returning, with work = None."""
    if not dist.is_initialized():
        return local, None
    world = dist.get_world_size(group)
    if not local.is_cuda or dist.get_backend(group) != "nccl" or n_total % world:
        return all_gather_rows(local, n_total, group), None
    lo, hi = shard_range(n_total, dist.get_rank(group), world)
    if local.shape[0] != hi - lo:
        raise ValueError(f"all_gather_rows_async: local shard has {local.shape[0]} rows, expected {hi - lo}")
    src = local.contiguous()
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    work = dist.all_gather_into_tensor(out, src, group=group, async_op=True)
    return out, work


def all_gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Gather per-rank row blocks (contiguous shards of n_total rows) into the full (n_total, ...) tensor.

    One all_gather_into_tensor moves everything.  Equal shards (the bench: B prompts per rank) gather straight
    into the result; ragged ones are padded to the largest shard and compacted afterwards.  Runs whenever a
    process group exists, world 1 included (the one-GPU RCCL rehearsal); without one it returns ``local``."""
    if not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    lo, hi = shard_range(n_total, dist.get_rank(group), world)
    if local.shape[0] != hi - lo:
        raise ValueError(f"all_gather_rows: local shard has {local.shape[0]} rows, expected {hi - lo}")
    per = -(-n_total // world)
    even = per * world == n_total
    src = local.contiguous()
    if not even:
        src = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        src[: local.shape[0]] = local
    out = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if local.is_cuda and dist.get_backend(group) != "nccl":  # gloo (device-map rehearsals): through the host
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(host, src.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, src, group=group)
    if even:
        return out
    rows = [out[r * per: r * per + (shard_range(n_total, r, world)[1] - shard_range(n_total, r, world)[0])]
            for r in range(world)]
    return torch.cat(rows, 0)


def generate_sharded(generate_fn: Callable[[int, int], torch.Tensor], n_total: int, group=None) -> torch.Tensor:
    """Run ``generate_fn(lo, hi) -> (hi-lo, N) waveforms`` on this rank's shard and all-gather the batch."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard_range(n_total, rank, world)
    local = generate_fn(lo, hi)
    return all_gather_rows(local, n_total, group)
