"""Multi-GPU frame sharding: one process per GPU, tile slabs gathered to rank 0.

The reference's render() (main.rs:159-290) runs num_cpus-2 workers that each
render whole 1-spp passes and merge them into the shared Image
(Image::merge, main.rs:629-638). Here the frame is split into 8x8 tiles
(tile t belongs to rank t % world, the rule mrt_render_args.shard_index /
shard_count apply inside the library); every rank accumulates ITS tiles in
sample order in its own HBM buffers, and publishing packs the rank's pixels
into a slab (16 B per pixel, mrt_shard_pack_device) and gathers the slabs
onto rank 0 (`dist.gather`: RCCL send/recv over xGMI with backend "nccl"),
which unpacks each into the published frame (mrt_shard_unpack_device).
Each rank sends only its own pixels: 16 B x W*H/N, i.e. 33.2 MB / N per
publish at 1080p, received by rank 0 as 33.2 MB in total.

Every pixel is summed on one rank only, so the published frame is
bit-identical to a single-GPU render of the same samples. Whether a bench
run is weak or strong scaling is the caller's choice of spp per step
(bench.py: weak by default).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


class ShardedFrame:
    """Per-rank accumulation of this rank's tiles + a slab gather per publish.

    `render_into(rgb, bounces, spp_begin, spp_count)` must accumulate samples
    [spp_begin, spp_begin+spp_count) of this rank's shard into the given
    buffers (float32 [H*W*3], int32 [H*W]) — `Context.render_device` on a GPU,
    the oracle in the CPU tests. With `ctx` (a massrt.Context) the slabs are
    packed and unpacked on the device by the library; without it (CPU
    tensors) by index gathers over the same pixel lists.
    """

    def __init__(self, width: int, height: int, device: torch.device, rank: int = 0, world: int = 1, ctx=None):
        import massrt

        self.W, self.H, self.rank, self.world, self.ctx = width, height, rank, world, ctx
        self.rgb = torch.zeros(width * height * 3, dtype=torch.float32, device=device)
        self.bounces = torch.zeros(width * height, dtype=torch.int32, device=device)
        self.spp = 0
        self._marks = []  # (start, end) CUDA events around each publish on a GPU
        if world == 1:
            self.out_rgb, self.out_bounces = self.rgb, self.bounces
            return
        self.pixels = [torch.from_numpy(massrt.shard_pixels(width, height, r, world).astype("int64")).to(device)
                       for r in range(world)]
        self.cap = max(int(p.numel()) for p in self.pixels)  # slabs padded to the largest shard
        self.slab = torch.zeros(self.cap * 4, dtype=torch.float32, device=device)
        if rank == 0:
            self.out_rgb = torch.zeros_like(self.rgb)
            self.out_bounces = torch.zeros_like(self.bounces)
            self.slabs = [torch.zeros_like(self.slab) for _ in range(world)]
        else:
            self.out_rgb = self.out_bounces = None
            self.slabs = None

    @property
    def slab_bytes(self) -> int:
        """Bytes each rank sends per publish (its own pixels, 16 B each)."""
        return 0 if self.world == 1 else int(self.pixels[self.rank].numel()) * 16

    def step(self, render_into: Callable[[torch.Tensor, torch.Tensor, int, int], None], spp_count: int,
             publish: bool = True):
        render_into(self.rgb, self.bounces, self.spp, spp_count)
        self.spp += spp_count
        if publish:
            self.publish()

    def _stream(self):
        return torch.cuda.current_stream().cuda_stream if self.rgb.is_cuda else None

    def _pack(self):
        if self.ctx is not None:
            self.ctx.shard_pack_device(self.W, self.H, self.rank, self.world, self.rgb.data_ptr(),
                                       self.bounces.data_ptr(), self.slab.data_ptr(), self._stream())
            return
        p = self.pixels[self.rank]
        s = self.slab.view(-1, 4)
        s[: p.numel(), :3] = self.rgb.view(-1, 3)[p]
        s[: p.numel(), 3] = self.bounces[p].view(torch.float32)

    def _unpack(self, r: int, slab: torch.Tensor):
        if self.ctx is not None:
            self.ctx.shard_unpack_device(self.W, self.H, r, self.world, slab.data_ptr(), self.out_rgb.data_ptr(),
                                         self.out_bounces.data_ptr(), self._stream())
            return
        p = self.pixels[r]
        s = slab.view(-1, 4)[: p.numel()]
        self.out_rgb.view(-1, 3)[p] = s[:, :3]
        self.out_bounces[p] = s[:, 3].contiguous().view(torch.int32)

    def publish(self):
        """Gather every rank's tile slab onto rank 0 (no-op for one rank)."""
        if self.world == 1:
            return
        timed = self.rgb.is_cuda
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        self._pack()
        if self.slab.is_cuda and dist.get_backend() == "gloo":  # gloo gathers host tensors (rehearsal/tests)
            torch.cuda.current_stream().synchronize()
            host = [torch.empty_like(self.slab, device="cpu") for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(self.slab.cpu(), host, dst=0)
            if self.rank == 0:
                for d, h in zip(self.slabs, host):
                    d.copy_(h)
        else:
            dist.gather(self.slab, self.slabs, dst=0)
        if self.rank == 0:
            for r, s in enumerate(self.slabs):
                self._unpack(r, s)
        if timed:
            e1.record()
            self._marks.append((e0, e1))

    def gather_ms(self, reset: bool = True) -> float:
        """Milliseconds the publishes since the last reset took on this rank's
        stream (pack + gather + unpack; a rank's gather includes waiting for
        the slowest rank)."""
        if not self._marks:
            return 0.0
        self._marks[-1][1].synchronize()
        t = sum(a.elapsed_time(b) for a, b in self._marks)
        if reset:
            self._marks = []
        return t

    def frame(self):
        """(rgb, bounces) of the whole image — valid on rank 0 after publish()."""
        return self.out_rgb, self.out_bounces

    def close(self):
        self.ctx = None
