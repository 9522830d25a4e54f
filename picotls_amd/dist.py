"""Multi-GPU plumbing for the record engine: one process per GPU, independent record shards, no data-path collective.

Record batches are embarrassingly parallel: every record is a self-contained AES-GCM computation, so
a node-level batch is split into contiguous record ranges, one per rank, each sealed/opened by an independent launch
on that rank's GPU. The only cross-rank traffic is a barrier around the timed region and a max/sum reduction of the
timings and byte counts (torch.distributed; "nccl" = RCCL on the GPU box, "gloo" in the CPU tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from .records import shard_ranges


def shard_for_rank(nrecs: int, rank: int, world: int, weights=None) -> tuple[int, int]:
    """Contiguous [begin, end) record range of `rank`; balanced by bytes when per-record weights are given
    (mixed-length batches), by count otherwise."""
    if weights is not None:
        return shard_ranges(weights, world)[rank]
    per = nrecs // world
    begin = rank * per
    end = nrecs if rank == world - 1 else begin + per
    return begin, end


@dataclass
class RankContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    dist: object = None
    device: object = None

    @classmethod
    def from_env(cls, backend: str = "nccl", device=None, always: bool = False) -> "RankContext":
        """The rank of this process (torch.distributed.run's environment). The process group (barrier, timing
        reductions) is joined when there are several ranks, or with `always` also for one (a one-GPU box can run the
        nccl branch that way)."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        ctx = cls(rank, world, local, None, device)
        if world > 1 or always:
            import torch.distributed as dist

            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group(backend)
            ctx.dist = dist
        return ctx

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.dist is None:
            return x
        import torch

        dev = self.device if (self.device is not None and self.dist.get_backend() == "nccl") else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, None if self.dist is None else self.dist.ReduceOp.MAX)

    def sum(self, x: float) -> float:
        return self._reduce(x, None if self.dist is None else self.dist.ReduceOp.SUM)

    def gather(self, values) -> list:
        """Every rank's `values` (a few numbers), in rank order, on every rank: a sum reduction of a world x k array in
        which each rank fills its own row (used to report the shards' record ranges; not a data-path collective)."""
        vals = [float(v) for v in values]
        if self.dist is None:
            return [vals]
        import torch

        dev = self.device if (self.device is not None and self.dist.get_backend() == "nccl") else "cpu"
        t = torch.zeros((self.world, len(vals)), dtype=torch.float64, device=dev)
        t[self.rank] = torch.tensor(vals, dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.cpu().tolist()

    @property
    def backend(self):
        return self.dist.get_backend() if self.dist is not None else None

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def aggregate_throughput(ctx: RankContext, payload_bytes: float, wall_s: float, steps: int) -> tuple[float, float]:
    """Whole-job seal+open GiB/s over all ranks: sum of payload bytes (sealed + opened) / max-over-ranks wall time."""
    total = ctx.sum(float(payload_bytes))
    wall = ctx.max(float(wall_s))
    return 2.0 * total * steps / wall / 2**30, wall


def shard_weights(lens: np.ndarray) -> np.ndarray:
    return np.asarray(lens, dtype=np.float64) + 64.0
