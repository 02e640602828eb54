"""Multi-GPU sharding of block batches: one process per GPU,
blocks dealt to ranks with no data-path collective.

JuiceFS compresses each 4 MiB block independently (pkg/chunk/cached_store.go
`upload` :356-398 / `load` :755-823 call the codec once per block), so a batch
of blocks partitions with no exchange step: rank r owns its own blocks and
torch.distributed (RCCL on the GPU box, gloo in the CPU tests) is used only for
the barrier around the timed region and the max-over-ranks / min-over-ranks
reductions of the timing and verification results.

The helpers here are backend-agnostic so that tests/test_shard_gloo.py runs the
exact code bench.py runs, with world_size 2 over gloo on the CPU.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, List, Sequence

import torch
import torch.distributed as dist


@dataclass
class RankEnv:
    world: int
    rank: int
    local: int


def rank_env() -> RankEnv:
    """torchrun's environment (RANK / LOCAL_RANK / WORLD_SIZE); 1 process when absent."""
    return RankEnv(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                   int(os.environ.get("LOCAL_RANK", "0")))


def seed_base(rank: int, nblk: int) -> int:
    """First synthetic-block seed of a rank: ranks generate disjoint block sets
    (seeds [1 + rank*nblk, 1 + (rank+1)*nblk)), so weak scaling decodes
    world*nblk distinct blocks."""
    return 1 + rank * nblk


def deal_round_robin(nblk: int, ndev: int) -> List[List[int]]:
    """Block indices per device for the batch ABI (jfs_*_batch, capi.hip
    `run_batch`): block i goes to device i % ndev, order kept."""
    if ndev < 1:
        raise ValueError("need at least one device")
    return [list(range(d, nblk, ndev)) for d in range(ndev)]


def _barrier(world: int) -> None:
    if world > 1:
        dist.barrier()


def timed_steps(step: Callable[[], None], steps: int, warmup: int, sync: Callable[[], None],
                world: int) -> float:
    """W untimed warmup steps, then EXACTLY `steps` timed steps bracketed by a
    barrier + device sync on both sides.  Returns this rank's wall seconds."""
    for _ in range(warmup):
        step()
    sync()
    _barrier(world)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    _barrier(world)
    return time.perf_counter() - t0


def max_over_ranks(x: float, world: int, device: torch.device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok: bool, world: int, device: torch.device) -> bool:
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item()) == 1


def whole_job_gib_s(world: int, nblk: int, block_bytes: int, steps: int, elapsed_s: float) -> float:
    """`value` of the bench line: uncompressed bytes all ranks produced in the
    timed steps over the slowest rank's wall time (weak scaling)."""
    return world * nblk * block_bytes * steps / elapsed_s / 2**30


def shard_sizes(sizes: Sequence[int], world: int) -> List[int]:
    """Total uncompressed bytes each rank owns under round-robin dealing."""
    out = [0] * world
    for i, s in enumerate(sizes):
        out[i % world] += int(s)
    return out
