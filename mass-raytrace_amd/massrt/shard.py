"""Multi-GPU frame sharding: one process per GPU, strong scaling.

The reference's render() (main.rs:159-290) runs num_cpus-2 workers that each
render whole 1-spp passes and merge them into the shared Image
(Image::merge, main.rs:629-638). Here the frame is split into 8x8 tiles
(tile t belongs to rank t % world, the same rule mrt_render_args.shard_index
/ shard_count apply inside the library), every rank accumulates ITS tiles in
sample order in its own HBM buffers, and after each step one
`dist.reduce(SUM)` of the per-rank frames publishes the image on rank 0.

Tiles are disjoint, so the reduce adds exact zeros: the published frame is
bit-identical to a single-GPU render of the same samples (the per-pixel sum
order never crosses ranks). This is the only exchange in the path; with
backend "nccl" it is one RCCL reduce over xGMI per step.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


class ShardedFrame:
    """Per-rank accumulation of this rank's tiles + one reduce per publish.

    `render_into(rgb, bounces, spp_begin, spp_count)` must accumulate samples
    [spp_begin, spp_begin+spp_count) of this rank's shard into the given
    buffers (float32 [H*W*3], int32 [H*W]) — `Context.render_device` on a GPU,
    the oracle in the CPU tests.
    """

    def __init__(self, width: int, height: int, device: torch.device, rank: int = 0, world: int = 1):
        self.W, self.H, self.rank, self.world = width, height, rank, world
        self.rgb = torch.zeros(width * height * 3, dtype=torch.float32, device=device)
        self.bounces = torch.zeros(width * height, dtype=torch.int32, device=device)
        if world > 1:
            self.out_rgb = torch.zeros_like(self.rgb)
            self.out_bounces = torch.zeros_like(self.bounces)
        else:
            self.out_rgb, self.out_bounces = self.rgb, self.bounces
        self.spp = 0

    def step(self, render_into: Callable[[torch.Tensor, torch.Tensor, int, int], None], spp_count: int,
             publish: bool = True):
        render_into(self.rgb, self.bounces, self.spp, spp_count)
        self.spp += spp_count
        if publish:
            self.publish()

    def publish(self):
        """Sum the per-rank tile frames onto rank 0 (no-op for one rank)."""
        if self.world == 1:
            return
        self.out_rgb.copy_(self.rgb)
        self.out_bounces.copy_(self.bounces)
        dist.reduce(self.out_rgb, 0, op=dist.ReduceOp.SUM)
        dist.reduce(self.out_bounces, 0, op=dist.ReduceOp.SUM)

    def frame(self):
        """(rgb, bounces) of the whole image — valid on rank 0 after publish()."""
        return self.out_rgb, self.out_bounces
