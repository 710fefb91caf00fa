"""Worker for tests/test_host.py::test_all_gather_two_ranks_gloo (launched by torch.distributed.run)."""
import torch
import torch.distributed as dist

from audiolcm_amd.distributed import (all_gather_rows_async, all_reduce_max, barrier, generate_sharded, init_from_env,
                                      shard_range)


def main():
    rank, world, _ = init_from_env("gloo")
    n = 5  # ragged: shards of 3 and 2

    def gen(lo, hi):
        # stand-in for the per-shard pipeline: row i is a deterministic function of prompt i only
        return torch.stack([torch.full((7,), float(i)) + torch.arange(7.0) for i in range(lo, hi)], 0)

    full = generate_sharded(gen, n)
    expect = torch.stack([torch.full((7,), float(i)) + torch.arange(7.0) for i in range(n)], 0)
    assert torch.equal(full, expect), (rank, full)
    lo, hi = shard_range(n, rank, world)
    assert hi - lo == (3 if rank == 0 else 2)
    assert all_reduce_max(0.5 + rank) == 0.5 + world - 1  # bench.py's max-over-ranks timing
    # bench.py's gather entry (async over RCCL; over gloo it completes before returning)
    lo, hi = shard_range(n, rank, world)
    full2, work = all_gather_rows_async(expect[lo:hi], n)
    assert work is None and torch.equal(full2, expect)
    barrier()
    if rank == 0:
        print("GATHER_OK")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
