"""Multi-GPU batch split: records are independent, so N GPUs of one
node each take a contiguous, equal-byte slice of the record array; there is no
collective on the data path.  torch.distributed (gloo) is used only as the control
plane: a barrier before/after the timed region and the max-over-ranks of the
elapsed time.  One process per GPU, launched by torch.distributed.run.
"""
from __future__ import annotations

import os

import numpy as np


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def device_for(local_rank: int, visible: int, allow_shared: bool | None = None) -> int:
    """GPU of a local rank.  Fewer visible GPUs than ranks is an error (a run
    asked for N GPUs must measure N, not wrap onto fewer), unless sharing is
    asked for explicitly: `allow_shared` or TLSGPU_ALLOW_SHARED_GPU=1 (the
    N-ranks-on-one-GPU rehearsal), which wraps."""
    if visible <= 0:
        raise RuntimeError("no GPU visible")
    if allow_shared is None:
        allow_shared = os.environ.get("TLSGPU_ALLOW_SHARED_GPU", "") == "1"
    if local_rank >= visible and not allow_shared:
        raise RuntimeError(f"local rank {local_rank} needs GPU {local_rank}, but only {visible} "
                           "visible (TLSGPU_ALLOW_SHARED_GPU=1 to share GPUs on purpose)")
    return local_rank % visible


def shard_by_bytes(lengths: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of the records rank `rank` owns: contiguous slices with balanced
    payload bytes (equal record counts when lengths are equal).  Cut k is the
    first record boundary whose byte prefix reaches k/world of the total, in
    exact integer arithmetic — the rule of the C ABI's tlsgpu_split_by_bytes."""
    n = len(lengths)
    if world <= 1:
        return 0, n
    csum = np.concatenate([[0], np.cumsum(lengths, dtype=np.int64)])
    total = int(csum[-1])
    cuts = [0] + [int(np.searchsorted(csum * world, total * k, side="left")) for k in
                  range(1, world)] + [n]
    return cuts[rank], cuts[rank + 1]


class ControlPlane:
    """Barrier and max-reduction across ranks (gloo, CPU tensors only)."""

    def __init__(self, world: int):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def max(self, values):
        if self.dist is None:
            return list(values)
        import torch
        t = torch.tensor(list(values), dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return [float(v) for v in t]

    def sum(self, values):
        if self.dist is None:
            return list(values)
        import torch
        t = torch.tensor(list(values), dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return [float(v) for v in t]

    def close(self) -> None:
        if self.dist is not None:
            self.dist.destroy_process_group()
