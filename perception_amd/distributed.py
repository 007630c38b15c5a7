"""Multi-GPU pose sharding and the argmin exchange.

One process per GPU.  The candidate-pose grid is split into contiguous global index ranges, every rank
scores its shard with no data-path collective, and the per-model selection keys
key = ((cost ^ 0x80000000) << 31) | global_index (int64, see include/pcore.h) are combined with ONE
all-reduce(MIN) -- RCCL over xGMI with the "nccl" backend on GPUs, gloo on CPU.  MIN over the keys is
exactly the reference's strict '<' first-index-wins scan (search_env.cpp:2560-2566).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) pose range of `rank` (remainder spread over the first ranks)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


# a one-rank process group (init_from_env(force=True) / PCORE_FORCE_PG=1): the exchange then runs even at world size 1,
# so the single-GPU bench can carry the collective in its loop and the RCCL path executes on a one-GPU box
_forced = False


def init_from_env(backend: str = None, force: Optional[bool] = None):
    """Initialise torch.distributed from torchrun's env (RANK / WORLD_SIZE / MASTER_*).  At world size 1 nothing is
    initialised unless `force` (default: PCORE_FORCE_PG=1), which starts a one-rank group on 127.0.0.1."""
    global _forced
    if force is None:
        force = os.environ.get("PCORE_FORCE_PG", "") == "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if dist.is_initialized() or (world <= 1 and not force):
        return
    if backend is None:
        # PCORE_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU (RCCL refuses
        # two ranks on one device); production multi-GPU runs use "nccl" = RCCL over xGMI
        backend = os.environ.get("PCORE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world <= 1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if "MASTER_PORT" not in os.environ:
            import socket

            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend, **kw)
    _forced = world <= 1


def exchange_active() -> bool:
    """Whether the argmin exchange runs: a process group of more than one rank, or a forced one-rank group."""
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _forced)


def allreduce_min_keys(keys: torch.Tensor) -> torch.Tensor:
    """In-place MIN all-reduce of the per-model int64 selection keys (no-op on one process)."""
    if exchange_active():
        dist.all_reduce(keys, op=dist.ReduceOp.MIN)
    return keys


def allreduce_min_keys_async(keys: torch.Tensor) -> Optional["dist.Work"]:
    """The same exchange, returned as a work handle (None on one process).  The caller waits on it before
    reading or rewriting `keys`; meanwhile the next batch's kernels run beside the collective (RCCL runs on
    its own stream, waiting only for the work already queued on the current one)."""
    if exchange_active():
        return dist.all_reduce(keys, op=dist.ReduceOp.MIN, async_op=True)
    return None
