"""Multi-GPU plumbing of the encode path: one process per GPU, one
independent H.264 stream per process (streams shard with no
data-path exchange, so there is no collective on the data; gloo carries the
barrier and the max-over-ranks of the wall time)."""
from __future__ import annotations

import os


def init_from_env():
    """Returns (rank, world_size, local_rank); joins the gloo group when
    launched by torchrun with more than one rank."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world, local


def world_size() -> int:
    """The process group's size (1 without a group)."""
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_initialized() else 1


def barrier():
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(value: float) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(value: float) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def sum_over_ranks(values):
    """Element-wise sum of a list of integers over the ranks."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return [int(v) for v in values]
    t = torch.tensor([int(v) for v in values], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]


def stream_seed(rank: int, base: int = 11) -> int:
    """Each rank encodes its own synthetic stream (weak scaling)."""
    return base + rank


def shutdown():
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
