"""One process per GPU: rank bookkeeping for tile-parallel runs.

rav1e parallelises a frame only across AV1 tiles (rayon `into_par_iter`
over `TileContextMut`s, src/encoder.rs:2772-2781); tiles share nothing but
read-only reference frames.  Here every rank (one per GPU, launched by
torch.distributed.run) owns its own tile stream, so the data path has no
collective: torch.distributed (gloo) carries only the start barrier and the
max-over-ranks time.  SURVEY.md §8e, DESIGN.md §6.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class RankInfo:
    rank: int
    world: int
    local_rank: int

    @property
    def frame_offset(self) -> int:
        """Synthetic-input time offset of this rank's tile stream: ranks
        encode different content (no two ranks redo the same work)."""
        return 1000 * self.rank


def rank_info() -> RankInfo:
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return RankInfo(rank, world, local)


class RankGroup:
    """torch.distributed on gloo (CPU tensors): barrier + reductions of
    scalars.  A no-op at world size 1."""

    def __init__(self, info: RankInfo, backend: str = "gloo"):
        self.info = info
        self.dist = None
        if info.world > 1:
            import torch.distributed as tdist
            if not tdist.is_initialized():
                tdist.init_process_group(backend, rank=info.rank, world_size=info.world)
            self.dist = tdist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, value: float) -> float:
        """Max over ranks (the bench's timed region is the slowest rank)."""
        if not self.dist:
            return float(value)
        import torch
        t = torch.tensor([float(value)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def gather_u64(self, value: int) -> list[int]:
        """Every rank's value (verification words), in rank order."""
        if not self.dist:
            return [int(value)]
        import torch
        t = torch.tensor([int(value) & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64)
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(self.info.world)]
        self.dist.all_gather(out, t)
        return [int(o[0]) for o in out]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()
            self.dist = None
