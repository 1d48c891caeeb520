#!/usr/bin/env python3
"""Headline benchmark: Msamples/s of the path-tracing hot path (BASELINE.json
metric) on BASELINE config 2 — SphereGrid (scenes/sphere_grid.rs, the
reference's random-spheres scene) at 1920x1080x1024spp, max depth 50.

A step = one pass of the hot path over one batch: `--spp-per-step` x N
samples (default 64 x N) of every pixel of the 1920x1080 frame; at N=1, 16
steps = the full 1024-spp config. With N GPUs (torchrun, one rank per GPU,
RCCL over xGMI) each rank renders every N-th 8x8 framebuffer tile of the same
frame, accumulating its tiles in its own HBM frame, and after every step the
per-rank frames are summed onto rank 0 with one dist.reduce
(massrt/shard.py; Image::merge, main.rs:629-638) — bit-identical to the
1-GPU image; no other exchange exists. Each rank's work per step is fixed
(2.07M/N pixels x 64N spp = 132.7M samples): "weak" scaling — a rank needs
that much in flight to keep its k_trace launches long compared with their
tails. `--strong` keeps 64 spp per step for any N instead.

Inputs (scene, BVH, camera) are resident in HBM before timing; the
accumulation buffers live in HBM. `value` = all samples of all ranks / the
max over ranks of the timed wall time.

roofline: dominant kernel k_trace (closest hit), HBM-bound by design
(no dense contraction). achieved = algorithmic bytes (SURVEY §8d model,
DESIGN.md §Roofline) per launch / average launch time, timed with HIP events
on the stream the kernels run on; peak 8000 GB/s (MI355X HBM3E spec).
traffic = FETCH_SIZE(x2, gfx950)+WRITE_SIZE per k_trace launch from the
committed rocprofv3 PMC summary for this config, else null.
cpu_baseline: the oracle's reference-mode restatement (main.rs:159-290
threading: num_cpus-2 workers rendering whole 1-spp passes) on a bounded row
band of the same frame, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mass-raytrace_amd"))

METRIC = "Msamples/sec (rays traced/sec) at 1920×1080×1024spp; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0

# SURVEY §8d algorithmic bytes of one k_trace segment (bytes per counted event)
TRACE_BYTES = {"node_visits": 32, "triangle_tests": 36, "sphere_tests": 16, "instance_entries": 48}
TRACE_RAY_BYTES = 32 + 16  # ray origin+direction read, hit record written


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="sphere_grid")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp-per-step", type=int, default=64, help="per GPU (x N frame spp per step) unless --strong")
    ap.add_argument("--strong", action="store_true", help="fixed spp per step for any N (strong scaling)")
    ap.add_argument("--total-spp", type=int, default=1024, help="spp of the config (reporting only)")
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--fused", action="store_true", help="one persistent k_render instead of the k_trace/k_shade loop")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--pmc-json", default=None, help="PMC summary (default profiles/pmc_<scene>.json)")
    return ap.parse_args()


def asset_dir(scene: str) -> Path:
    if scene.startswith("mesh") or scene.startswith("menger"):
        sys.path.insert(0, str(REPO / "tools"))
        from gen_assets import ensure_assets
        return ensure_assets(REPO / "assets", mesh=scene.startswith("mesh"), textures=scene.endswith("textured"),
                             environment=scene.startswith("menger"))
    return REPO / "tests" / "golden"


def cpu_baseline(scene: str, W: int, H: int, max_depth: int, seconds: float, seed: int):
    import oracle  # CPU restatement (test infrastructure): the baseline, never the product
    import massrt

    share = min(16, os.cpu_count() or 4)  # the box's CPU share for one GPU
    threads = max(1, share - 2)  # render(): num_cpus - 2 workers (main.rs:159-160)
    o = oracle.Scene(1).builtin(scene, float(massrt.ASPECT_RATIO), str(asset_dir(scene)))
    r0 = H // 2 - 4
    secs, _, _ = o.bench_reference_mode(W, H, 1, seed=seed + 7, max_depth=max_depth, threads=threads,
                                        row_begin=r0, row_end=r0 + 8)
    rate = threads * W * 8 / max(secs, 1e-6)
    rows = int(max(8, min(H, seconds * rate / (threads * W))))
    r0 = max(0, H // 2 - rows // 2)
    secs, _, _ = o.bench_reference_mode(W, H, 1, seed=seed + 8, max_depth=max_depth, threads=threads,
                                        row_begin=r0, row_end=r0 + rows)
    samples = threads * W * rows
    return {
        "value": round(samples / secs / 1e6, 4),
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{scene} {W}x{H}, rows [{r0},{r0 + rows}) x {threads} workers x 1 pass (1 spp each) = "
                   f"{samples} samples in {secs:.1f}s; oracle reference mode (recursive virtual traversal, "
                   f"main.rs:159-290 threading), g++ -O3 scalar"),
    }


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import massrt
    from massrt.shard import ShardedFrame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(a.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    W, H = a.width, a.height
    spp = a.spp_per_step if a.strong else a.spp_per_step * world

    ctx = massrt.Context(torch.cuda.current_device())
    b = massrt.Builder(1).builtin(a.scene, float(massrt.ASPECT_RATIO), str(asset_dir(a.scene)))
    ctx.upload(b)
    frame = ShardedFrame(W, H, dev, rank, world)
    stream = torch.cuda.current_stream().cuda_stream

    def step(counters=False, timing=False):
        def render_into(rgb, bounces, s0, n):
            args = ctx.args(W, H, s0, n, a.seed, a.max_depth, rank, world, counters=counters, time_kernels=timing,
                            flags=massrt.RENDER_FUSED if a.fused else 0)
            ctx.render_device(args, rgb.data_ptr(), bounces.data_ptr(), stream)

        frame.step(render_into, spp)  # renders this rank's tiles, then one reduce onto rank 0

    # warmup; the first warmup step also counts traversal events (statistics
    # for the algorithmic-bytes model — not part of the timed region)
    ctx.reset_counters()
    for k in range(a.warmup):
        step(counters=(k == 0))
    torch.cuda.synchronize()
    cnt = ctx.counters()
    ctx.reset_kernel_stats()

    timing = not a.no_kernel_timing
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(timing=timing)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ks = ctx.kernel_stats()

    samples_total = W * H * spp * a.steps
    value = samples_total / elapsed / 1e6

    # roofline of k_trace on this rank
    roof = None
    if timing and cnt["samples"] > 0 and ks["trace_launches"] > 0:
        seg_per_sample = cnt["segments"] / cnt["samples"]
        bytes_per_seg = (sum(TRACE_BYTES[k] * cnt[k] for k in TRACE_BYTES) / max(cnt["segments"], 1)
                         + TRACE_RAY_BYTES)
        segs = seg_per_sample * (samples_total / world)  # this rank's share of the timed samples
        achieved = bytes_per_seg * segs / (ks["trace_ms"] * 1e-3) / 1e9
        traffic = None
        pmc = Path(a.pmc_json) if a.pmc_json else REPO / "profiles" / f"pmc_{a.scene}.json"
        if pmc.exists():
            try:
                pj = json.loads(pmc.read_text())
                if pj.get("width") == W and pj.get("height") == H:
                    traffic = pj.get("k_trace_hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "k_trace", "bytes_per_launch": round(bytes_per_seg * segs / ks["trace_launches"]),
            "avg_launch_ms": round(ks["trace_ms"] / ks["trace_launches"], 4),
            "launches": int(ks["trace_launches"]), "bytes_per_segment": round(bytes_per_seg, 1),
            "segments_per_sample": round(seg_per_sample, 4),
            "lane_utilisation": round(cnt["lane_steps"] / max(cnt["wave_slots"], 1), 4),
        }

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(a.scene, W, H, a.max_depth, a.cpu_seconds, a.seed)
        except Exception as e:  # baseline failure must not hide the GPU number
            cpu = {"value": None, "error": str(e)}

    if rank == 0:
        mean_bounces = float(frame.frame()[1].double().sum().item()) / (W * H * spp * (a.steps + a.warmup))
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if (a.strong and world > 1) else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (built-in scene, fixed seeds)",
            "config": {
                "workload": f"{a.scene} {W}x{H}x{a.total_spp}spp, max_depth {a.max_depth}",
                "scene": a.scene, "width": W, "height": H, "spp_per_step": spp,
                "samples_per_step": W * H * spp, "max_depth": a.max_depth,
                "parallelism": f"tile-shard x{world}" + (
                    (" + RCCL reduce" if a.dist_backend == "nccl" else f" + {a.dist_backend} reduce") if world > 1 else ""),
                "mean_bounces_per_sample": round(mean_bounces, 4),
                "mrays_per_s": round(value * (roof["segments_per_sample"] if roof else float("nan")), 1),
            },
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if cpu and cpu.get("value"):
            line["config"]["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
