"""One process per GPU: rank bookkeeping and the tile-parallel encode of one
stream.

rav1e parallelises a frame only across AV1 tiles (rayon `into_par_iter`
over `TileContextMut`s, src/encoder.rs:2772-2781); tiles share nothing but
the reference frames.  Here every rank (one per GPU, launched by
torch.distributed.run) codes one tile group of every frame of the SAME
stream; after each frame the reconstruction of every group must reach every
rank before the next frame's motion search (the reference's write-back,
src/encoder.rs:3411-3429): an all-gather of the packed group regions --
RCCL over xGMI inside rv_replay_frame on the GPU, gloo in the CPU tests.
torch.distributed (gloo) also carries the barrier, the max-over-ranks time
and the RCCL bootstrap.  SURVEY.md §8e, DESIGN.md §6.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


@dataclass
class RankInfo:
    rank: int
    world: int
    local_rank: int


def rank_info() -> RankInfo:
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return RankInfo(rank, world, local)


class RankGroup:
    """torch.distributed on gloo (CPU tensors): barrier, reductions of
    scalars, byte all-gathers.  A no-op at world size 1."""

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

    def all_gather_bytes(self, buf: np.ndarray, size: int) -> list[np.ndarray]:
        """Every rank's byte buffer (padded to `size`), in rank order."""
        if not self.dist:
            return [buf]
        import torch
        t = torch.zeros(size, dtype=torch.uint8)
        t[: buf.size] = torch.from_numpy(buf)
        out = [torch.zeros(size, dtype=torch.uint8) for _ in range(self.info.world)]
        self.dist.all_gather(out, t)
        return [o.numpy() for o in out]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()
            self.dist = None


class TileParallel:
    """This rank's share of a tile-parallel encode: the engine (HipReplay or
    the oracle's CpuReplay) codes tile group rects[my] of every frame; frame()
    also moves every group's reconstruction to every rank.

    * HipReplay with an RCCL communicator: rv_replay_frame packs the group,
      all-gathers over RCCL on the replay stream, unpacks and pads -- no
      host round trip (comm from rav1e_amd.replay.RcclComm).
    * CpuReplay: pack, gloo all-gather, unpack, pad."""

    def __init__(self, engine, rects, my, group: RankGroup, comm=None):
        self.engine, self.rects, self.my, self.group = engine, list(rects), my, group
        self.world = len(self.rects)
        self.host = not hasattr(engine, "set_groups")
        if self.world > 1 and not self.host:
            if comm is None:
                raise ValueError("a GPU engine in a multi-rank run needs an RCCL communicator")
            engine.set_groups(self.rects, my, comm.h)
            if getattr(engine, "imp_window", 0):
                # the importance window: every group's lookahead part is
                # all-gathered with the same communicator, on the encode's
                # stream, before the frames whose window needs it
                engine.set_la_exchange(comm=comm.h)
        if self.host:
            self.size = max(engine.region_bytes(r) for r in self.rects)

    def _lookahead_parts(self):
        """A group's importance window (CpuReplay): every lookahead frame the
        next frame needs, each group's part all-gathered and imported (the
        propagation reads the whole frame)."""
        due = self.engine.la_due() if hasattr(self.engine, "la_due") else None
        if due is None:
            return
        nxt, last, _ = due
        size = max(self.engine.la_part_bytes(r) for r in self.rects)
        mine_b = self.engine.la_part_bytes(self.rects[self.my])
        for m in range(nxt, last + 1):
            mine = self.engine.la_group(m, mine_b)
            bufs = self.group.all_gather_bytes(mine, size)
            for k, (rect, b) in enumerate(zip(self.rects, bufs)):
                if k != self.my:
                    self.engine.la_import(m, rect, b[: self.engine.la_part_bytes(rect)])

    def frame(self):
        if self.world == 1:
            return self.engine.frame()
        if not self.host:
            return self.engine.frame()
        self._lookahead_parts()
        info = self.engine.frame(pad=False)
        mine = self.engine.export(self.rects[self.my])
        bufs = self.group.all_gather_bytes(mine, self.size)
        for k, (rect, b) in enumerate(zip(self.rects, bufs)):
            if k != self.my:
                self.engine.import_(rect, b[: self.engine.region_bytes(rect)])
        self.engine.pad_recon()
        return info

    def results(self):
        return self.engine.results()

    def entropy_stats(self):
        return self.engine.entropy_stats()
