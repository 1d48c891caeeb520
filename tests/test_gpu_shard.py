"""Multi-rank GPU path on one MI355X: two processes (gloo for the gather,
both ranks on device 0) render their 8x8 tiles with the product kernels into
massrt.shard.ShardedFrame, which packs each rank's pixels into a slab on the
device (mrt_shard_pack_device), gathers the slabs to rank 0 and unpacks them
there (mrt_shard_unpack_device) — the bench's N>1 path (bench.py,
Image::merge main.rs:629-638) below RCCL. Rank 0's published frame must be
bit-identical to a one-rank render of the same samples.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]
W, H, SPP, STEPS = 131, 75, 2, 3  # ragged: tiles cut by both frame edges


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir, scene):
    for p in (REPO, REPO / "mass-raytrace_amd"):
        sys.path.insert(0, str(p))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import massrt
        from massrt.shard import ShardedFrame

        torch.cuda.set_device(0)
        ctx = massrt.Context(0)
        b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(REPO / "tests" / "golden"))
        ctx.upload(b)
        dev = torch.device("cuda", 0)
        # gloo: ShardedFrame stages the device slabs through host memory for the gather
        frame = ShardedFrame(W, H, dev, rank, world, ctx=ctx)
        stream = torch.cuda.current_stream().cuda_stream

        def render_into(rgb, bounces, s0, n):
            ctx.render_device(ctx.args(W, H, s0, n, 9, 50, rank, world), rgb.data_ptr(), bounces.data_ptr(), stream)

        for _ in range(STEPS):
            frame.step(render_into, SPP)
        torch.cuda.synchronize()
        if rank == 0:
            rgb, bo = frame.frame()
            np.save(Path(out_dir) / "rgb.npy", rgb.cpu().numpy())
            np.save(Path(out_dir) / "b.npy", bo.cpu().numpy().view(np.uint32))
        with open(Path(out_dir) / f"slab{rank}.txt", "w") as f:
            f.write(str(frame.slab_bytes))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gpu_frame_matches_one_rank(ctx, golden_dir, tmp_path, world):
    import massrt

    scene = "sphere_grid"
    mp.spawn(_rank, args=(world, _free_port(), str(tmp_path), scene), nprocs=world, join=True)
    b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), golden_dir)
    ctx.upload(b)
    acc = (np.zeros(W * H * 3, np.float32), np.zeros(W * H, np.uint32))
    for k in range(STEPS):
        acc = ctx.render(W, H, k * SPP, SPP, seed=9, accum=acc)
    assert np.array_equal(np.load(tmp_path / "b.npy"), acc[1])
    assert np.array_equal(np.load(tmp_path / "rgb.npy").view(np.uint32), acc[0].view(np.uint32))
    # each rank sent only its own pixels
    sent = sum(int((tmp_path / f"slab{r}.txt").read_text()) for r in range(world))
    assert sent == W * H * 16


def test_shard_pack_unpack_roundtrip(ctx):
    import massrt

    Wp, Hp, n = 70, 41, 3
    dev = torch.device("cuda", 0)
    rgb = torch.rand(Wp * Hp * 3, device=dev)
    bo = torch.randint(0, 1 << 30, (Wp * Hp,), dtype=torch.int32, device=dev)
    out_rgb, out_b = torch.zeros_like(rgb), torch.zeros_like(bo)
    for r in range(n):
        px = massrt.shard_pixels(Wp, Hp, r, n)
        slab = torch.zeros(max(px.size, 1) * 4, device=dev)
        ctx.shard_pack_device(Wp, Hp, r, n, rgb.data_ptr(), bo.data_ptr(), slab.data_ptr())
        ctx.shard_unpack_device(Wp, Hp, r, n, slab.data_ptr(), out_rgb.data_ptr(), out_b.data_ptr())
        torch.cuda.synchronize()
        s = slab.view(-1, 4)[: px.size].cpu()
        pt = torch.from_numpy(px.astype(np.int64))
        assert torch.equal(s[:, :3], rgb.view(-1, 3).cpu()[pt])
        assert torch.equal(s[:, 3].contiguous().view(torch.int32), bo.cpu()[pt])
    assert torch.equal(out_rgb, rgb) and torch.equal(out_b, bo)


def test_cpp_multi_device_driver_matches_one_device(ctx, golden_dir, tmp_path):
    """examples/mrt_render_multi.cpp (one process, one context per device,
    slabs gathered with peer copies) on devices 0,0,0 — three shards on the
    one GPU here — writes the one-device image: raw sums bit-exact. (Its RCCL
    transport needs distinct devices and is not exercised on a 1-GPU box.)"""
    import subprocess

    import massrt

    exe = Path(massrt.__file__).parent / "mrt_render_multi"
    Wc, Hc, passes = 100, 57, 3
    raw = tmp_path / "frame.raw"
    r = subprocess.run([str(exe), "cube_field", str(Wc), str(Hc), str(passes), str(tmp_path / "m.png"),
                        str(golden_dir), "0,0,0", "peer", str(raw)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    b = massrt.Builder(1).builtin("cube_field", float(massrt.ASPECT_RATIO), golden_dir)
    ctx.upload(b)
    rgb, bo = ctx.render(Wc, Hc, 0, passes, seed=1)
    data = np.fromfile(raw, dtype=np.uint32)
    assert np.array_equal(data[: Wc * Hc * 3], rgb.view(np.uint32))
    assert np.array_equal(data[Wc * Hc * 3:], bo)
