"""Multi-rank sharding path (massrt/shard.py, used by bench.py --gpus N) on
CPU ranks over gloo: each rank accumulates its 8x8 tiles, one slab gather per step
publishes the frame on rank 0. The oracle stands in for the GPU renderer
here (test infrastructure only); the GPU tests cover the device side of the
same shard_index/shard_count arguments.

Expected: the published frame is bit-identical to a single-rank render of
the same samples (every pixel is summed on one rank only).
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

REPO = Path(__file__).resolve().parents[1]
W, H, SPP, STEPS = 40, 24, 2, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_scene():
    import massrt
    import oracle
    return oracle.Scene(1).builtin("cornell", float(massrt.ASPECT_RATIO), str(REPO / "tests" / "golden"))


def _rank(rank, world, port, out_dir):
    for p in (REPO, REPO / "mass-raytrace_amd"):
        sys.path.insert(0, str(p))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from massrt.shard import ShardedFrame
        o = _oracle_scene()
        frame = ShardedFrame(W, H, torch.device("cpu"), rank, world)

        def render_into(rgb, bounces, s0, n):
            o.render(W, H, s0, n, seed=3, shard_index=rank, shard_count=world, threads=1,
                     accum=(rgb.numpy(), bounces.numpy().view(np.uint32)))

        for _ in range(STEPS):
            frame.step(render_into, SPP)
        if rank == 0:
            rgb, b = frame.frame()
            np.save(Path(out_dir) / "rgb.npy", rgb.numpy())
            np.save(Path(out_dir) / "b.npy", b.numpy().view(np.uint32))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frame_matches_single_rank(tmp_path, world):
    mp.spawn(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    o = _oracle_scene()
    rgb = np.zeros(W * H * 3, np.float32)
    b = np.zeros(W * H, np.uint32)
    for k in range(STEPS):  # single rank, same per-step accumulation
        o.render(W, H, k * SPP, SPP, seed=3, threads=2, accum=(rgb, b))
    assert np.array_equal(np.load(tmp_path / "b.npy"), b)
    assert np.array_equal(np.load(tmp_path / "rgb.npy"), rgb)
    assert b.sum() > 0
