"""Multi-GPU sharding of the NDT + PointNet path.

Clouds are independent from preprocessing through the forward, so a batch of
``total`` clouds is split into contiguous shards, one process per GPU
(torchrun / torch.distributed.run; backend "nccl" is RCCL on ROCm), with no
collective on the data path.  The only collectives are the timing barrier,
the max-over-ranks of the elapsed time, and -- when a caller wants the global
result -- an all-gather of the per-rank outputs (C4: 16 x 1000 x 29 fp32 =
1.9 MB per rank).

The reference has no multi-GPU path for this (tools/train.py runs one
process); the layout here follows SURVEY §8e: throughput = all clouds / max
over ranks of the rank time ("weak" scaling: per-GPU work fixed as N grows).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def world_from_env() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) as torch.distributed.run exports them."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str, device: Optional[torch.device] = None) -> bool:
    """Joins the process group when WORLD_SIZE > 1 (env:// rendezvous; use
    MASTER_ADDR=127.0.0.1).  Returns whether a group is active."""
    _, _, world = world_from_env()
    if world <= 1:
        return False
    if not dist.is_initialized():
        kw = {"device_id": device} if (device is not None and device.type == "cuda") else {}
        dist.init_process_group(backend, **kw)
    return True


def shard(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard (start, count) of ``total`` clouds for ``rank``; the
    first ``total % world`` ranks take one extra cloud."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _reduce_device() -> torch.device:
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(value: float) -> float:
    """The maximum of ``value`` over all ranks (the job's wall time)."""
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_reduce_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float) -> float:
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_reduce_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_shards(out: torch.Tensor) -> torch.Tensor:
    """Concatenates every rank's ``[b_r, ...]`` output along dim 0 in rank
    order (shards may differ in size by one cloud)."""
    if not dist.is_initialized():
        return out
    world = dist.get_world_size()
    dev = _reduce_device()
    n = torch.tensor([out.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes)
    buf = torch.zeros((cap,) + tuple(out.shape[1:]), dtype=out.dtype, device=dev)
    buf[: out.shape[0]] = out.to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
