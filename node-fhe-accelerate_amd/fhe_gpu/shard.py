"""Batch sharding across GPUs.

Polynomials are independent: every op on the path (NTT, polymul, modmul,
external product) shards by contiguous polynomial ranges with NO exchange
during compute.  One process per GPU (torch.distributed, RCCL over xGMI);
the only collective is the optional final gather of results to rank 0.

``shard_range`` is the partition; ``run_sharded`` applies an op to this rank's
shard; ``gather_to_root`` collects the shards (``dist.gather`` on the
process group -- RCCL for GPU tensors, gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Callable, Sequence, Tuple


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of ``total`` items for ``rank``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def run_sharded(op: Callable, inputs: Sequence, rank: int, world: int):
    """Apply ``op`` to this rank's slice (leading dim = batch) of each input."""
    total = inputs[0].shape[0]
    lo, hi = shard_range(total, rank, world)
    return op(*[x[lo:hi] for x in inputs])


def gather_to_root(local, total: int, rank: int, world: int, group=None):
    """Gather per-rank shards (``local``: torch tensor, leading dim = this
    rank's shard) into one tensor on rank 0 (None elsewhere).  Shards may be
    ragged; they are padded to the largest shard for the collective."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    sizes = [shard_range(total, r, world) for r in range(world)]
    mx = max(hi - lo for lo, hi in sizes)
    pad = local
    if local.shape[0] < mx:
        pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad.contiguous(), gather_list=bufs, dst=0, group=group)
    if rank != 0:
        return None
    return torch.cat([b[: hi - lo] for b, (lo, hi) in zip(bufs, sizes)], dim=0)
