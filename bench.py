#!/usr/bin/env python3
"""Headline benchmark: Msamples/s of the path-tracing hot path (BASELINE.json
metric) on BASELINE config 2 — SphereGrid (scenes/sphere_grid.rs, the
reference's random-spheres scene) at 1920x1080x1024spp, max depth 50 — plus,
in the same invocation, north_star's target scene (config 4's 1M-triangle
binary PLY mesh, `mesh_ply`) as `config.secondary`.

A step = one pass of the hot path over one batch: `--spp-per-step` (default
1024) samples of every pixel of the 1920x1080 frame, i.e. the whole
1024-spp config frame, for ANY number of GPUs ("strong" scaling: BASELINE's
metric and config 4 fix the frame, 1920x1080x1024 spp, and split it over
1/2/4/8 GPUs; `--weak` renders 1024 x N spp per step instead).

With N GPUs (`--gpus N`, default mode "multi") ONE process drives all N
devices through the library's multi-device context — the boundary a Rust
render() links (mrt_create_multi + mrt_image_*, include/massrt.h; main.rs:
159-170): every device renders every N-th 8x8 framebuffer tile of the frame
into its own HBM, one host thread per device, and at the end of every step
the library gathers the devices' tile slabs onto device 0 (Image::merge,
main.rs:629-638) with RCCL send/recv over xGMI (peer copies on repeated
devices, e.g. `--devices 0,0` to rehearse on one GPU) — bit-identical to the
1-GPU image. Under a launcher (torch.distributed.run --nproc-per-node N)
rank 0 is that process and ranks 1..N-1 only join the barriers around the
timed region (they never touch a GPU). `--mode ranks` is the alternative:
one process per GPU, each rendering its tiles through mrt_render_device on
torch's stream, slabs gathered with torch.distributed (massrt/shard.py).

Inputs (scene, BVH, camera) are resident in HBM before timing; the
accumulation buffers live in HBM. `value` = all samples rendered / the max
over ranks of the timed wall time (barrier + device sync on both sides).

roofline (dominant kernel k_trace, closest hit):
  achieved = algorithmic bytes per launch (SURVEY §8d model: 32 B per box,
             36 per triangle, 16 per sphere, 48 per instance entry, 48 per
             ray in/out) / the average k_trace launch time measured with HIP
             events on the launch stream. The record stream is served from
             L1/L2 (and the Infinity Cache for the 1M-triangle mesh), so the
             peak it is priced against is the cache path's: L2 36.9 TB/s with
             L1 reuse (MI355X_MICROARCH.md §L2) — never the HBM peak.
  hbm      = measured HBM bytes per launch (rocprofv3 PMC, (2*FETCH_SIZE +
             WRITE_SIZE) KiB, gfx950 x2 read correction) / rocprof's average
             launch time, against 8 TB/s. From profiles/pmc_<scene>.json,
             used only when its stamp (scene, size, spp per step, source
             hash) matches this run; else null.
  bound    = the unit the PMC counters show busiest (TA/L1 address path, HBM,
             VALU), e.g. "l1/ta" for SphereGrid.
roofline_k_shade: k_shade (path-state streaming) against HBM: per shaded
  path the state read and the survivor's state or the finished result
  written, plus the shading data of each closest hit and the texels
  (shade_bytes), with the PMC traffic/limiter of the same stamped profile
  and the waves' material coherence (ABI v9 counters).
cpu_baseline: the oracle's reference-mode restatement (main.rs:159-290
threading: num_cpus-2 workers rendering whole 1-spp passes) on a stratified
sample of rows spread over the whole frame, rank 0 at N=1 only, plus an
all-logical-cores run; host model and core counts are recorded;
gpu_over_cpu is against the whole host (host_estimate when the job has a
CPU quota), gpu_over_cpu_quota<N> against the job's share.
config.dropin: the Rust binding's render() call pattern (massrt.render:
pre-pass, clear, num_cpus-2 passes per frame in batches of 256 into the
device-resident image, a tonemap + host copy per batch), 1080p, both scenes.
--gpus N without a launcher starts N ranks itself (torch.distributed.run).
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
N_CU, N_XCD = 256, 8  # MI355X: 256 CUs in 8 XCDs (MI355X_MICROARCH.md)
# record stream bandwidth is cache-served: L2 aggregate with L1 reuse (MI355X_MICROARCH.md §L2)
CACHE_PEAK_GBS = 36900.0

# SURVEY §8d algorithmic bytes of one k_trace segment (bytes per counted event)
TRACE_BYTES = {"node_visits": 32, "triangle_tests": 36, "sphere_tests": 16, "instance_entries": 48}
TRACE_RAY_BYTES = 32 + 16  # ray origin+direction read, hit record written

# k_shade's algorithmic bytes, from the counting
# step's events: every shaded path reads its state (ro, rd, thr, rng: 4 x 16 B)
# and hit record (16 B); a survivor writes its state to the next pool (4 x 16
# B), a finished sample its 16-B result; every closest hit reads the shading
# data of its primitive (§8d: 36 B normals + 24 B uv + 32 B material) and
# every texel tap (counted per texel) 4 B of RGBA8. rad moves only for the
# rare path that holds radiance (a Mix that emits and scatters): not counted.
SHADE_READ_PATH, SHADE_WRITE_SURVIVOR, SHADE_WRITE_RESULT = 4 * 16 + 16, 4 * 16, 16
SHADE_HIT, SHADE_TEXEL = 36 + 24 + 32, 4


def shade_bytes(cnt) -> dict:
    """k_shade's algorithmic read and write bytes over the counted step."""
    shaded, finished = cnt.get("shaded", 0), min(cnt.get("samples", 0), cnt.get("shaded", 0))
    reads = SHADE_READ_PATH * shaded + SHADE_HIT * cnt.get("closest_hits", 0) + SHADE_TEXEL * cnt.get("texel_taps", 0)
    writes = SHADE_WRITE_SURVIVOR * (shaded - finished) + SHADE_WRITE_RESULT * finished
    return {"reads": reads, "writes": writes, "total": reads + writes}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="sphere_grid")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp-per-step", type=int, default=1024, help="frame spp per step (x N with --weak)")
    ap.add_argument("--weak", action="store_true", help="spp-per-step x N per step (weak scaling); default strong")
    ap.add_argument("--mode", choices=("multi", "ranks"), default="multi",
                    help="multi: one process, one multi-device context (library gather); ranks: a process per GPU")
    ap.add_argument("--devices", default=None, help="multi mode: device ordinals, e.g. 0,0 to rehearse on one GPU")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="context option (mrt_set_option), repeatable")
    ap.add_argument("--total-spp", type=int, default=1024, help="spp of the config (reporting only)")
    ap.add_argument("--no-configs", action="store_true", help="skip the BASELINE config 3 / 5 lines (config.c3/c5)")
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target length of each CPU baseline run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--secondary", default="mesh_ply", help="second scene of the same run ('' or 'none': off)")
    ap.add_argument("--secondary-steps", type=int, default=2)
    ap.add_argument("--fused", action="store_true", help="one persistent k_render instead of the k_trace/k_shade loop")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--pmc-json", default=None, help="PMC summary (default profiles/pmc_<scene>.json)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in render() call-pattern runs")
    ap.add_argument("--dropin-batch", type=int, default=256, help="1-spp passes per mrt_image_render call")
    return ap.parse_args()


def src_hash() -> str:
    """Hash of the library sources (tools/src_hash.py): a PMC profile is valid
    only for the code it measured, and the loaded library must carry it."""
    sys.path.insert(0, str(REPO / "tools"))
    from src_hash import src_hash as h

    return h()


def launch_plan(gpus: int, env: dict, argv: list, port: int, mode: str = "multi"):
    """How `bench.py --gpus N` runs: None = this process runs in place (the
    only process, or one rank of a launcher's job); else the command that
    starts N ranks (mode "ranks": torch.distributed.run, one process per GPU,
    rendezvous on 127.0.0.1). Mode "multi" never spawns: one process drives
    every device. A launcher's WORLD_SIZE must agree with --gpus."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}: the launcher and the flag disagree")
        return None
    if gpus <= 1 or mode == "multi":
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def asset_dir(scene: str, rank: int = 0, world: int = 1) -> Path:
    if scene.startswith("mesh") or scene.startswith("menger"):
        sys.path.insert(0, str(REPO / "tools"))
        from gen_assets import ensure_assets

        kw = dict(mesh=scene.startswith("mesh"), textures=scene.endswith("textured"),
                  environment=scene.startswith("menger"))
        if world > 1:  # one writer per node, the others wait for it
            import torch.distributed as dist
            if rank == 0:
                ensure_assets(REPO / "assets", **kw)
            dist.barrier()
        return ensure_assets(REPO / "assets", **kw)
    return REPO / "tests" / "golden"


def host_info() -> dict:
    model, phys = "unknown", set()
    try:
        cur = {}
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if ":" not in line:
                if cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, v = (s.strip() for s in line.split(":", 1))
            cur[k] = v
            if k == "model name":
                model = v
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "physical_cores": len(phys) or None,
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota}


def cpu_baseline(scene: str, W: int, H: int, max_depth: int, seconds: float, seed: int) -> dict:
    """The reference's render() threading (main.rs:159-160: num_cpus - 2 worker
    threads, each rendering whole 1-spp passes into a private buffer merged
    under a mutex, main.rs:235-290) over a stratified sample of rows spread
    over the whole frame, then the same rows with every logical CPU."""
    import oracle  # CPU restatement (test infrastructure): the baseline, never the product
    import massrt

    host = host_info()
    logical = host["logical_cpus"] or 1
    ref_threads = max(1, logical - 2)
    o = oracle.Scene(1).builtin(scene, float(massrt.ASPECT_RATIO), str(asset_dir(scene)))

    def run(threads, n_rows, sd):
        step = max(1, H // n_rows)
        r0 = step // 2
        secs, _, _ = o.bench_reference_mode(W, H, 1, seed=sd, max_depth=max_depth, threads=threads,
                                            row_begin=r0, row_end=H, row_step=step)
        rows = len(range(r0, H, step))
        return secs, rows, step, r0

    secs, rows, _, _ = run(ref_threads, 4, seed + 7)  # calibration
    rate = ref_threads * W * rows / max(secs, 1e-6)
    n_rows = int(max(4, min(H, seconds * rate / (ref_threads * W))))
    secs, rows, step, r0 = run(ref_threads, n_rows, seed + 8)
    samples = ref_threads * W * rows
    value = samples / secs / 1e6
    secs_all, rows_all, _, _ = run(logical, n_rows, seed + 9)
    value_all = logical * W * rows_all / secs_all / 1e6
    quota = host["cgroup_cpu_quota"]
    cpus_avail = min(host["affinity_cpus"] or logical, int(quota) if quota else logical)
    out = {
        "value": round(value, 4),
        "unit": "Msamples/s",
        # the reference's num_cpus-2 threads run on the CPUs this job may use
        "cores": cpus_avail,
        "threads": ref_threads,
        "cpus_available": cpus_avail,
        "host_physical_cores": host["physical_cores"],
        "kind": "port",
        "all_cores": {"value": round(value_all, 4), "threads": logical, "seconds": round(secs_all, 2)},
        "host": host,
        "sample": (f"{scene} {W}x{H}: rows {r0}, {r0 + step}, ... ({rows} rows, every {step}th, whole frame) x "
                   f"{ref_threads} workers (num_cpus-2, main.rs:159-160) x 1 pass (1 spp each) = {samples} samples "
                   f"in {secs:.1f}s; oracle reference mode (recursive virtual traversal, main.rs:159-290 "
                   f"threading), g++ -O3 scalar"),
    }
    if quota and quota < logical:
        # This job may use only `quota` CPUs of the host, so the runs above are
        # quota-bound. Measure the rate per CPU with exactly that many workers
        # and scale it to every logical CPU of the host: an estimate (it assumes
        # SMT siblings scale like cores — generous to the CPU), not a measurement.
        q = max(1, int(quota))
        secs_q, rows_q, _, _ = run(q, n_rows, seed + 10)
        per_cpu = W * rows_q / secs_q / 1e6  # q workers x 1 pass each, over q CPUs
        out["host_estimate"] = {
            "value": round(per_cpu * logical, 3), "per_cpu": round(per_cpu, 4), "threads_measured": q,
            "basis": f"job CPU quota {quota} of {logical} logical CPUs: rate of {q} workers / {q} x {logical} "
                     f"(linear in logical CPUs; an estimate, not measured)"}
    return out


def c1_runs(a) -> dict:
    """BASELINE config 1: SphereGrid (the reference's random-spheres scene,
    sphere_grid.rs:23-94) at 400x225x64 spp, whole frame — the reference-mode
    CPU run (min(num_cpus-2, 64) workers x whole 1-spp passes = 64 passes,
    main.rs:159-290) and the same 64 spp on the GPU."""
    import torch

    import massrt
    import oracle

    W, H, spp = 400, 225, 64
    threads = max(1, min((os.cpu_count() or 1) - 2, spp))
    o = oracle.Scene(1).builtin("sphere_grid", float(massrt.ASPECT_RATIO), str(REPO / "tests" / "golden"))
    secs, _, _ = o.bench_reference_mode(W, H, spp // threads, seed=a.seed, max_depth=a.max_depth, threads=threads)
    cpu_samples = W * H * threads * (spp // threads)
    ctx = massrt.Context(torch.cuda.current_device())
    b = massrt.Builder(1).builtin("sphere_grid", float(massrt.ASPECT_RATIO), str(REPO / "tests" / "golden"))
    ctx.upload(b)
    b.close()
    ctx.render(W, H, 0, 4, seed=a.seed)  # warm up
    t0 = time.perf_counter()
    ctx.render(W, H, 0, spp, seed=a.seed)  # host buffers in and out (the whole mrt_render call)
    gsecs = time.perf_counter() - t0
    ctx.close()
    return {"workload": f"sphere_grid {W}x{H}x{spp}spp (BASELINE config 1)",
            "cpu": {"value": round(cpu_samples / secs / 1e6, 4), "unit": "Msamples/s", "seconds": round(secs, 2),
                    "threads": threads, "passes_per_thread": spp // threads, "kind": "port"},
            "gpu": {"value": round(W * H * spp / gsecs / 1e6, 2), "unit": "Msamples/s", "seconds": round(gsecs, 4),
                    "note": "one mrt_render call incl. host copies; too small to fill the GPU"}}


def dropin_run(a, scene: str, headline: float | None) -> dict:
    """The drop-in render() call pattern (bindings/rust/src/lib.rs `render`,
    restated as massrt.render): one frame of the reference's render()
    (main.rs:150-295) at frame_limit 1 — pre-pass, Image::clear, then
    num_cpus-2 workers x 1 pass each = that many 1-spp passes (main.rs:159-160,
    243-280), run --dropin-batch passes per mrt_image_render call into the
    device-resident image, and after every batch the update the reference's
    UI gets (UserEvent::Update -> to_rgb_bytes): the display bytes tone-mapped
    on the GPU and copied to the host. Timed: the whole render() call."""
    import torch

    import massrt

    W, H = a.width, a.height
    ctx = massrt.Context(torch.cuda.current_device())
    b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(asset_dir(scene)))
    ctx.upload(b)
    b.close()
    img = massrt.Image(ctx, W, H)
    workers = massrt.default_workers()
    st = massrt.SampleStreams(a.seed)
    last = {}

    def update(im, passes):  # the UI's redraw: display bytes on the host
        last["bytes"] = im.tonemap()
        last["passes"] = passes

    massrt.render(img, st, frame_limit=1, workers=min(workers, 2 * a.dropin_batch), batch=a.dropin_batch,
                  update=update)  # warm-up frame (untimed)
    t0 = time.perf_counter()
    n = massrt.render(img, st, frame_limit=1, workers=workers, batch=a.dropin_batch, update=update)
    secs = time.perf_counter() - t0
    assert last["passes"] == n == workers
    img.close()
    ctx.close()
    value = W * H * n / secs / 1e6
    return {"workload": f"{scene} {W}x{H}, render(frame_limit=1): {workers} workers (num_cpus-2) x 1 pass",
            "value": round(value, 2), "unit": "Msamples/s", "seconds": round(secs, 3), "passes": n,
            "batch": a.dropin_batch, "updates": -(-n // a.dropin_batch),
            "of_headline": round(value / headline, 3) if headline else None,
            "includes": "pre-pass, clear, every batch's render and tonemap + 6 MB device-to-host copy"}


def load_pmc(path: Path, stamp: dict):
    """PMC summary for this exact configuration and source, else None."""
    if not path.exists():
        return None
    try:
        pj = json.loads(path.read_text())
    except (OSError, ValueError):
        return None
    st = {"n_gpus": 1, "traversal": 0, **pj.get("stamp", {})}  # profiles are taken on one GPU, the reference walk unless stamped
    if any(st.get(k) != v for k, v in stamp.items()):
        return None
    return pj


def limiter(pj: dict, kernel: str = "k_trace"):
    """Utilisation of the units `kernel` can be bound by, from the PMC summary."""
    k = pj.get("kernels", {}).get(kernel, {})
    out = {}
    avg_ns = k.get("avg_ns")
    if k.get("hbm_bytes_per_launch") and avg_ns:
        out["hbm"] = k["hbm_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9 / HBM_PEAK_GBS
    for name in ("ta_busy", "valu_busy", "l1_hit", "l2_hit", "wait_frac", "lds_busy"):
        if k.get(name) is not None:
            out[name] = k[name]
    return out


def context_options(a) -> dict:
    """MASSRT_OPTIONS (massrt.env_options), then --opt NAME=VALUE on top: the
    options bench.py's contexts are created with (mrt_set_option)."""
    import massrt

    out = massrt.env_options()
    out.update(massrt.parse_options(",".join(a.opt), "--opt"))
    return out


def step_plan(a, n_gpus: int) -> dict:
    """What one timed step renders with n_gpus GPUs: the whole --spp-per-step
    frame (strong scaling: BASELINE's 1920x1080x1024spp frame split over the
    GPUs), or spp-per-step x N with --weak. The workload label names exactly
    that."""
    spp = a.spp_per_step * (n_gpus if a.weak else 1)
    return {"spp_per_step": spp, "samples_per_step": a.width * a.height * spp,
            "scaling": "weak" if (a.weak and n_gpus > 1) else "strong",
            "workload": f"{a.scene} {a.width}x{a.height}x{spp}spp per step, max_depth {a.max_depth}"}


def device_list(a) -> list:
    """Multi mode: the devices of the one context (--devices, else 0..N-1)."""
    if a.devices:
        devs = [int(x) for x in a.devices.split(",") if x.strip()]
        if len(devs) != a.gpus:
            raise SystemExit(f"bench.py: --devices lists {len(devs)} devices but --gpus {a.gpus}")
        return devs
    return list(range(a.gpus))


class MultiRunner:
    """One process, one context over `devices` (mrt_create_multi) and a
    device-resident Image: a step renders the frame's samples on every
    device (each its tiles) and gathers the tiles onto device 0 (library
    RCCL send/recv or peer copies) — what a Rust render() over several GPUs
    calls (bindings/rust/src/lib.rs)."""

    def __init__(self, a, scene, devices):
        import massrt

        self.a, self.devices, self.W, self.H = a, devices, a.width, a.height
        self.ctx = massrt.Context(devices=devices, options=context_options(a))
        t = time.perf_counter()
        b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(asset_dir(scene)))
        self.ctx.upload(b)
        b.close()
        self.t_load = time.perf_counter() - t
        self.img = massrt.Image(self.ctx, self.W, self.H)
        self.next_sample = 0
        self.gathers = (0, 0.0)

    def step(self, spp, counters=False, timing=False):
        self.img.render(self.a.seed, self.next_sample, spp, self.a.max_depth, counters=counters, time_kernels=timing)
        self.next_sample += spp
        self.img.gather()  # Image::merge onto device 0; returns once every device's work has ended

    def sync(self):
        self.img.gather()

    def reset_gather_stats(self):
        self.gathers = self.img.gather_stats()
        self.dev_ms = self.img.device_stats()

    def gather_stats(self):
        b, ms = self.img.gather_stats()
        return b - self.gathers[0], ms - self.gathers[1]

    def device_ms(self):
        """Per-device render ms since reset_gather_stats (HIP events)."""
        return [x - y for x, y in zip(self.img.device_stats(), self.dev_ms)]

    def mean_bounces(self):
        _, b, passes = self.img.read()
        return float(b.astype("float64").sum()) / (self.W * self.H * max(passes, 1))

    def close(self):
        self.img.close()
        self.ctx.close()


class RankRunner:
    """--mode ranks: this process renders its tiles on its own GPU through
    mrt_render_device on torch's stream; slabs gathered with torch.distributed
    (massrt/shard.py)."""

    def __init__(self, a, scene, rank, world, dev):
        import torch

        import massrt
        from massrt.shard import ShardedFrame

        self.a, self.rank, self.world, self.W, self.H = a, rank, world, a.width, a.height
        self.ctx = massrt.Context(torch.cuda.current_device(), options=context_options(a))
        t = time.perf_counter()
        b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(asset_dir(scene, rank, world)))
        self.ctx.upload(b)
        b.close()
        self.t_load = time.perf_counter() - t
        self.frame = ShardedFrame(self.W, self.H, dev, rank, world, ctx=self.ctx)
        self.stream = torch.cuda.current_stream().cuda_stream
        self.steps = 0

    def step(self, spp, counters=False, timing=False):
        import massrt

        def render_into(rgb, bounces, s0, n):
            args = self.ctx.args(self.W, self.H, s0, n, self.a.seed, self.a.max_depth, self.rank, self.world,
                                 counters=counters, time_kernels=timing,
                                 flags=massrt.RENDER_FUSED if self.a.fused else 0)
            self.ctx.render_device(args, rgb.data_ptr(), bounces.data_ptr(), self.stream)

        self.frame.step(render_into, spp)  # renders this rank's tiles, then gathers the tile slabs onto rank 0
        self.steps += 1

    def sync(self):
        import torch

        torch.cuda.synchronize()

    def reset_gather_stats(self):
        self.frame.gather_ms()

    def gather_stats(self):
        return self.frame.slab_bytes, self.frame.gather_ms()

    def mean_bounces(self):
        spp = self.frame.spp
        return float(self.frame.frame()[1].double().sum().item()) / (self.W * self.H * max(spp, 1))

    def close(self):
        self.frame.close()
        self.ctx.close()


def verify_gather(a, r, scene: str, devices, spp: int = 4) -> dict:
    """N > 1, multi mode: outside the timed region, a
    fresh image on the bench's own multi-device context renders `spp`
    samples of the whole frame and gathers them onto device 0 over the
    context's transport; a one-device context on devices[0] renders the same
    (seed, samples). Each pixel is summed in sample order on one device, so
    the two must be bit-identical."""
    import numpy as np

    import massrt

    img = massrt.Image(r.ctx, r.W, r.H)
    try:
        img.render(a.seed, 0, spp, a.max_depth)
        img.gather()
        rgb, bounces, passes = img.read()
    finally:
        img.close()
    one = massrt.Context(devices[0], options=context_options(a))
    try:
        b = massrt.Builder(1).builtin(scene, float(massrt.ASPECT_RATIO), str(asset_dir(scene)))
        one.upload(b)
        b.close()
        orgb, ob = one.render(r.W, r.H, 0, spp, seed=a.seed, max_depth=a.max_depth)
    finally:
        one.close()
    same_rgb = bool(np.array_equal(rgb.view(np.uint32), orgb.view(np.uint32)))
    same_b = bool(np.array_equal(bounces, ob))
    return {"identical": same_rgb and same_b and passes == spp, "rgb_bits_equal": same_rgb,
            "bounces_equal": same_b, "spp": spp, "pixels": r.W * r.H,
            "against": f"one-device context on device {devices[0]}, same seed and samples",
            "differing_pixels": int((bounces != ob).sum() + (rgb != orgb).reshape(-1, 3).any(1).sum())}


def timed_region(world, steps_fn, sync_fn, pg_dev=None):
    """Barrier + device sync on both sides of `steps_fn`; every rank's wall
    time, and the job's = the slowest rank's."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    sync_fn()
    t0 = time.perf_counter()
    steps_fn()
    sync_fn()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_rank = [elapsed]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        if pg_dev is not None:
            t = t.to(pg_dev)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        per_rank = [float(p[0]) for p in parts]
    return max(per_rank), per_rank


def roofline_for(a, scene, cnt, ks, samples_total, elapsed, n_gpus, plan, trav: int = 0) -> tuple:
    """(roofline of k_trace, roofline_k_shade) from the counting warmup step's
    event counts and the timed steps' HIP-event kernel times."""
    if not (cnt["samples"] > 0 and ks["trace_launches"] > 0):
        return None, None
    seg_per_sample = cnt["segments"] / cnt["samples"]
    bytes_per_seg = (sum(TRACE_BYTES[k] * cnt[k] for k in TRACE_BYTES) / max(cnt["segments"], 1) + TRACE_RAY_BYTES)
    segs = seg_per_sample * samples_total  # every device's share of the timed samples (kernel stats sum over them)
    # traversal launches: k_trace, plus the drain hand-off's fused k_render
    # launches (render.hip launch_finish_v), which trace the last paths'
    # segments — their shading time counts too (conservative)
    fin_ms, fin_n = ks.get("finish_ms", 0.0), int(ks.get("finish_launches", 0))
    trav_launches = ks["trace_launches"] + fin_n
    bytes_per_launch = bytes_per_seg * segs / trav_launches
    avg_ms = (ks["trace_ms"] + fin_ms) / trav_launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    import massrt

    # the walk the run used (`trav`, the context's tuning): its own profile,
    # profiles/pmc_<scene>_nf.json for the near-first walk
    stamp = {"scene": scene, "width": a.width, "height": a.height, "spp_per_step": plan["spp_per_step"],
             "src": src_hash(), "n_gpus": n_gpus, "traversal": trav}
    tag = "_nf" if trav else ""
    pmc_path = (Path(a.pmc_json) if (a.pmc_json and scene == a.scene and not trav)
                else REPO / "profiles" / f"pmc_{scene}{tag}.json")
    pj = load_pmc(pmc_path, stamp)
    pmc_basis = "this configuration"
    if pj is None and n_gpus > 1:
        # N > 1: each device runs the 1-GPU kernels on its shard of the tiles,
        # so the N=1 profile of the same source, scene and frame stands for the
        # per-device limiter (labelled; traffic per launch is not rescaled)
        pj = load_pmc(pmc_path, {**stamp, "n_gpus": 1})
        if pj is not None:
            pmc_basis = "the N=1 profile of the same source and config, as each device's limiter (not re-measured at N)"
    lim = limiter(pj) if pj else {}
    traffic = pj["kernels"]["k_trace"].get("hbm_bytes_per_launch") if (pj and pmc_basis == "this configuration") else None
    bound = "unmeasured (no PMC profile of this source and config)"
    if lim:  # the busiest unit; none at half its peak: the dependent record loads' latency binds
        cand = {"l1/ta": lim.get("ta_busy", 0.0), "hbm": lim.get("hbm", 0.0), "valu": lim.get("valu_busy", 0.0)}
        bound = max(cand, key=cand.get)
        if cand[bound] < 0.5:
            bound = "latency (dependent record loads)"
    roof = {
        "bound": bound, "achieved": round(achieved, 1), "peak": CACHE_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / CACHE_PEAK_GBS, 4), "traffic": round(traffic) if traffic else None,
        "peak_source": "record stream is L1/L2-served: L2 36.9 TB/s with L1 reuse, MI355X_MICROARCH.md §L2",
        "hbm": ({"achieved": round(lim["hbm"] * HBM_PEAK_GBS, 1), "peak": HBM_PEAK_GBS,
                 "frac": round(lim["hbm"], 4)} if "hbm" in lim else None),
        "limiter": {k: round(v, 4) for k, v in lim.items()} or None,
        "pmc": str(pmc_path.relative_to(REPO)) + f" (src {stamp['src']})" if pj else None,
        "pmc_basis": pmc_basis if pj else None,
        "kernel": "k_trace + drain k_render<adopt>", "bytes_per_launch": round(bytes_per_launch),
        "avg_launch_ms": round(avg_ms, 4), "launches": int(trav_launches),
        "k_trace": {"launches": int(ks["trace_launches"]),
                    "avg_launch_ms": round(ks["trace_ms"] / ks["trace_launches"], 4)},
        "finish": ({"launches": fin_n, "avg_launch_ms": round(fin_ms / fin_n, 4)} if fin_n else None),
        "achieved_per_step": round(bytes_per_seg * segs / elapsed / 1e9, 1),
        "bytes_per_segment": round(bytes_per_seg, 1), "segments_per_sample": round(seg_per_sample, 4),
        "lane_utilisation": round(cnt["lane_steps"] / max(cnt["wave_slots"], 1), 4),
        # box tests the early slab decision left to the exact test (path.h box_hit_any)
        "box_exact_frac": round(cnt.get("box_exact", 0) / max(cnt["node_visits"], 1), 5),
        # near-first walk (option traversal=1): segments whose hit check sent
        # them back to the reference's walk (path.h nf_finish)
        "vnf_fallback_frac": round(cnt.get("vnf_fallbacks", 0) / max(cnt["segments"], 1), 6),
    }
    # what a walk costs per unit of traversal work: frac
    # prices algorithmic bytes, so a walk that needs fewer bytes reads lower
    # at the same speed; CU time per segment and per box test rank walks by
    # speed. From the HIP-event launch times (always) and, with a matching PMC
    # profile, from its cycle counters (GRBM_GUI_ACTIVE over the 8 XCDs = the
    # launch's clocks; TA_TA_BUSY_sum = address-unit cycles summed over CUs).
    segs_per_launch = segs / trav_launches
    visits_per_launch = cnt["node_visits"] / max(cnt["segments"], 1) * segs_per_launch
    cu_ns = avg_ms * 1e6 * N_CU
    roof["work_rate"] = {
        "box_tests_per_segment": round(cnt["node_visits"] / max(cnt["segments"], 1), 2),
        "cu_ns_per_segment": round(cu_ns / segs_per_launch, 2),
        "cu_ns_per_box_test": round(cu_ns / max(visits_per_launch, 1), 3),
        "basis": "HIP-event launch time x 256 CUs / (counted box tests or segments per launch); "
                 "NF node records count as 2 box tests"}
    kt = (pj or {}).get("kernels", {}).get("k_trace", {}) if pmc_basis == "this configuration" else {}
    if kt.get("GRBM_GUI_ACTIVE_units") and kt.get("pmc_launches"):
        clocks = kt["GRBM_GUI_ACTIVE_units"] / N_XCD  # per launch (pmc_summary.py averages per launch)
        roof["work_rate"]["cu_cycles_per_box_test"] = round(clocks * N_CU / max(visits_per_launch, 1), 2)
        roof["work_rate"]["cu_cycles_per_segment"] = round(clocks * N_CU / segs_per_launch, 1)
        if kt.get("TA_TA_BUSY_sum"):
            roof["work_rate"]["ta_cycles_per_box_test"] = round(kt["TA_TA_BUSY_sum"] / max(visits_per_launch, 1), 2)
        roof["work_rate"]["pmc"] = "profiles/" + pmc_path.name
    shade = None
    if cnt.get("shaded") and ks["shade_launches"] > 0:
        # k_shade: HBM-streaming (path state in and out, shading data, texels): shade_bytes()
        sbc = shade_bytes(cnt)
        scale = samples_total / max(cnt["samples"], 1) / ks["shade_launches"]  # counted step -> one timed launch
        sb = sbc["total"] * scale
        sms = ks["shade_ms"] / ks["shade_launches"]
        shade = {"kernel": "k_shade", "bound": "hbm", "bytes_per_launch": round(sb), "avg_launch_ms": round(sms, 4),
                 "launches": int(ks["shade_launches"]), "achieved": round(sb / (sms * 1e-3) / 1e9, 1),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(sb / (sms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "reads_per_launch": round(sbc["reads"] * scale), "writes_per_launch": round(sbc["writes"] * scale),
                 "bytes_per_path": round(sbc["total"] / max(cnt["shaded"], 1), 1),
                 "paths_per_sample": round(cnt["shaded"] / max(cnt["samples"], 1), 4)}
        if cnt.get("shade_waves"):  # ABI v9: how material-coherent a shading wave is
            shade["coherence"] = {"kinds_per_wave": round(cnt["shade_kinds"] / cnt["shade_waves"], 3),
                                  "materials_per_wave": round(cnt["shade_materials"] / cnt["shade_waves"], 3),
                                  "note": "distinct material kinds (a miss = one more) and material indices among "
                                          "a k_shade wave's lanes, counting step; a material-sorted pool could bring "
                                          "both to ~1"}
        # the same kernel with ONE queue (option queues=1 profile, tools/profile.sh TAG=_solo): alone on the
        # GPU; in the bench run it shares the CUs with the other queue's k_trace by design
        pjs = load_pmc(REPO / "profiles" / f"pmc_{scene}_solo.json", stamp)
        kso = pjs["kernels"].get("k_shade", {}) if pjs else {}
        if kso.get("hbm_bytes_per_launch") and kso.get("avg_ns"):
            shade["solo"] = {"pmc": f"profiles/pmc_{scene}_solo.json (src {stamp['src']}, queues=1)",
                             "avg_launch_ms": round(kso["avg_ns"] * 1e-6, 4),
                             "traffic": round(kso["hbm_bytes_per_launch"]),
                             "achieved": round(kso["hbm_bytes_per_launch"] / kso["avg_ns"], 1),
                             "frac": round(kso["hbm_bytes_per_launch"] / kso["avg_ns"] / HBM_PEAK_GBS, 4)}
        ksh = pj["kernels"].get("k_shade", {}) if pj else {}
        if ksh.get("hbm_bytes_per_launch"):  # PMC of the same source and config (rocprof's per-launch average)
            shade["traffic"] = round(ksh["hbm_bytes_per_launch"])
            shade["traffic_over_algorithmic"] = round(ksh["hbm_bytes_per_launch"] / max(sb, 1), 3)
            if ksh.get("FETCH_SIZE") is not None and ksh.get("WRITE_SIZE") is not None:
                shade["traffic_reads"] = round(2 * ksh["FETCH_SIZE"] * 1024)  # x2: gfx950 FETCH_SIZE (pmc_summary.py)
                shade["traffic_writes"] = round(ksh["WRITE_SIZE"] * 1024)
            shade["pmc_avg_launch_ms"] = round(ksh["avg_ns"] * 1e-6, 4)
            shade["limiter"] = {k: round(v, 4) for k, v in limiter(pj, "k_shade").items()}
    # north_star asks >= 40% of HBM peak during BVH traversal: the co-run and
    # solo HBM fractions of k_trace from the stamped PMC profiles, side by side
    pjt = load_pmc(REPO / "profiles" / f"pmc_{scene}_solo.json", stamp)
    solo = limiter(pjt).get("hbm") if pjt else None
    roof["north_star_hbm_traversal"] = {
        "co_run": round(lim["hbm"], 4) if "hbm" in lim else None, "solo": round(solo, 4) if solo else None,
        "target": 0.40, "met": bool(lim.get("hbm", 0) >= 0.40 or (solo or 0) >= 0.40),
        "reason": "the record stream is cache-resident (L1 hit %s, L2 hit %s): traversal reads its algorithmic "
                  "bytes from L1/L2, which exceed the HBM peak; HBM carries only misses and the path state"
                  % (round(lim["l1_hit"], 3) if "l1_hit" in lim else "?", round(lim["l2_hit"], 3) if "l2_hit" in lim else "?")}
    return roof, shade


def run_scene(a, scene: str, steps: int, warmup: int, rank: int, world: int, dev, cpu: bool, devices=None,
              spp=None, width=None, height=None) -> dict:
    """Bench one scene: `warmup` untimed steps (the first counts traversal
    events for the algorithmic-bytes model), then `steps` timed steps."""
    import copy

    a = copy.copy(a)
    a.scene = scene
    if spp is not None:
        a.spp_per_step = spp
    if width:
        a.width, a.height = width, height
    W, H = a.width, a.height
    n_gpus = len(devices) if devices is not None else world
    plan = step_plan(a, n_gpus)
    spp = plan["spp_per_step"]
    r = MultiRunner(a, scene, devices) if devices is not None else RankRunner(a, scene, rank, world, dev)
    for k in range(max(1, warmup)):
        r.step(spp, counters=(k == 0))
    r.sync()
    cnt = r.ctx.counters()
    r.ctx.reset_kernel_stats()
    r.reset_gather_stats()  # drop the warmup publishes
    timing = not a.no_kernel_timing
    pg_dev = dev if (devices is None and world > 1 and a.dist_backend == "nccl") else None

    def steps_fn():
        for _ in range(steps):
            r.step(spp, timing=timing)

    elapsed, per_rank = timed_region(world, steps_fn, r.sync, pg_dev)
    g_bytes, g_ms = r.gather_stats()
    ks = r.ctx.kernel_stats()
    samples_total = W * H * spp * steps
    value = samples_total / elapsed / 1e6
    roof, shade = (None, None)
    if timing:
        # ranks mode: this rank's share of the samples and its own launches
        share = samples_total / (world if devices is None else 1)
        roof, shade = roofline_for(a, scene, cnt, ks, share, elapsed, n_gpus, plan,
                                   int(r.ctx.tuning().get("traversal", 0)))
    out = {"scene": scene, "value": round(value, 3), "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps,
           "warmup": warmup, "width": W, "height": H, "spp_per_step": spp, "samples_per_step": W * H * spp,
           "workload": plan["workload"], "scaling": plan["scaling"], "n_gpus": n_gpus,
           "scene_load_s": round(r.t_load, 2), "roofline": roof, "roofline_k_shade": shade,
           "tuning": r.ctx.tuning()}
    if n_gpus > 1:
        if devices is not None:
            out["gather"] = {"path": "one process: mrt_create_multi + mrt_image_render / mrt_image_gather",
                             "devices": devices, "transport": r.ctx.transport(),
                             "bytes_to_device0_per_step": round(g_bytes / steps),
                             "ms_per_step": round(g_ms / steps, 3),
                             "device_render_ms_per_step": [round(x / steps, 3) for x in r.device_ms()],
                             "per_rank_ms_per_step": [round(e / steps * 1e3, 3) for e in per_rank]}
            try:
                out["gather"]["check"] = verify_gather(a, r, scene, devices)
                out["gather"]["identical"] = out["gather"]["check"]["identical"]
            except Exception as e:  # a failed check must not hide the timed number
                out["gather"]["check"] = {"identical": None, "error": str(e)}
                out["gather"]["identical"] = None
        else:
            out["gather"] = {"path": "one process per GPU: mrt_render_device + torch.distributed gather",
                             "transport": "RCCL (dist.gather over xGMI)" if a.dist_backend == "nccl" else
                             f"{a.dist_backend} (host-staged)", "bytes_per_rank_per_step": g_bytes,
                             "bytes_to_rank0_per_step": W * H * 16,
                             "per_rank_ms_per_step": [round(e / steps * 1e3, 3) for e in per_rank]}
    if rank == 0:
        out["mean_bounces_per_sample"] = round(r.mean_bounces(), 4)
        out["mrays_per_s"] = round(value * roof["segments_per_sample"], 1) if roof else None
    r.close()
    if cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(scene, W, H, a.max_depth, a.cpu_seconds, a.seed)
        except Exception as e:  # baseline failure must not hide the GPU number
            out["cpu_baseline"] = {"value": None, "error": str(e)}
        cb = out["cpu_baseline"]
        if cb.get("host_estimate"):
            # the whole host (every logical CPU; estimated from the quota-bound rate)
            out["gpu_over_cpu"] = round(value / cb["host_estimate"]["value"], 1)
            out["gpu_over_cpu_basis"] = "whole host (host_estimate, all logical CPUs)"
            if cb.get("value"):
                out[f"gpu_over_cpu_quota{cb['cpus_available']}"] = round(value / cb["value"], 1)
        elif cb.get("value"):
            out["gpu_over_cpu"] = round(value / cb["value"], 1)
            out["gpu_over_cpu_basis"] = f"measured on {cb['cpus_available']} CPUs (the whole host)"
    return out


def idle_rank(world: int, n_scenes: int):
    """Multi mode under a launcher: ranks 1..N-1 own no GPU work (rank 0's
    context drives every device); they join each timed region's barriers and
    report their wall time, so the job's time is still the max over ranks."""
    for _ in range(n_scenes):
        timed_region(world, lambda: None, lambda: None)


def config_lines(a, rank, world, dev, devices) -> dict:
    """BASELINE configs 3 and 5 on one GPU, each with
    its roofline: cube_field 1080p x 1024 spp (one frame per step) and the
    textured 1M-triangle mesh + environment map at 4K, 256 spp per step (of
    the config's 4096: 2.12G samples, one results chunk)."""
    out = {}
    for key, scene, kw, label in (
            ("c3", "cube_field", dict(spp=1024), "BASELINE config 3: cube.ply x 10k instances, 1080p x 1024 spp"),
            ("c5", "mesh_obj_textured", dict(spp=256, width=3840, height=2160),
             "BASELINE config 5: textured 1M-tri mesh + env map, 4K, 256 of 4096 spp per step")):
        try:
            r = run_scene(a, scene, 2 if key == "c5" else 1, 1, rank, world, dev, False, devices, **kw)
            r["config"] = label
            out[key] = r
        except Exception as e:
            out[key] = {"error": str(e)}
    return out


WALK_NAMES = {0: "reference", 1: "near_first"}


def other_walk_lines(a, rank, world, dev, devices, runs: dict) -> dict:
    """Each workload of the line (headline, secondary, config 3) again with
    the other walk (massrt.h MRT_TRAVERSAL_*): the default (AUTO) takes the
    proven near-first walk where it is faster (sphere_grid, cube_field) and
    the reference's left-first walk elsewhere (mesh_ply, Menger), so the line
    carries both numbers for every scene. Both walks return the reference's
    closest hits."""
    import copy

    out = {"exactness": "both walks return the reference's closest hits: the reference walk by construction, the "
                        "near-first walk by the rounding bound of DESIGN.md §4 (slab_check bound checks, GPU parity)"}
    for key, scene, steps, kw in (("headline", a.scene, 2, {}), ("secondary", a.secondary, 2, {}),
                                  ("c3", "cube_field", 1, dict(spp=1024))):
        used = runs.get(key)
        if not scene or scene == "none" or not used or "value" not in used:
            continue
        walk = int(used.get("tuning", {}).get("traversal", 0))
        other = 1 - walk
        b = copy.copy(a)
        b.opt = list(a.opt) + [f"traversal={other}"]
        try:
            r = run_scene(b, scene, steps, 1, rank, world, dev, False, devices, **kw)
            got = int(r["tuning"].get("traversal", 0))
            out[key] = {"scene": scene, "walk_used": WALK_NAMES[walk], "value_used": used["value"],
                        "other_walk": WALK_NAMES[got], "other_value": r["value"],
                        "used_over_other": round(used["value"] / r["value"], 3) if r["value"] else None,
                        "ms_per_step": r["ms_per_step"], "steps": steps,
                        "vnf_fallback_frac": (r["roofline"] or {}).get("vnf_fallback_frac"),
                        "k_trace_avg_launch_ms": ((r["roofline"] or {}).get("k_trace") or {}).get("avg_launch_ms")}
            if got == walk:
                out[key]["note"] = "the scene has no near-first trees: one walk only"
        except Exception as e:
            out[key] = {"error": str(e)}
    return out


def main():
    a = parse()
    # --gpus N without a launcher in "ranks" mode: start the N ranks ourselves,
    # before anything here touches a GPU, and exit with their status (rank 0
    # prints the line). "multi" mode always runs in this process.
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = launch_plan(a.gpus, os.environ, sys.argv[1:], port, a.mode)
    if cmd is not None:
        import subprocess

        sys.exit(subprocess.call(cmd, env=dict(os.environ)))

    import datetime

    import torch
    import torch.distributed as dist

    import massrt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    multi = a.mode == "multi"
    devices = device_list(a) if multi else None
    n_gpus = len(devices) if multi else world
    secondary = a.secondary if (a.secondary and a.secondary != "none" and a.secondary != a.scene) else None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # multi mode: the launcher's other ranks only join barriers (gloo, no GPU)
        backend = "gloo" if multi else a.dist_backend
        if not multi:
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend, timeout=datetime.timedelta(hours=2))
        if multi and rank != 0:
            idle_rank(world, 1 + (secondary is not None))
            dist.destroy_process_group()
            return
    if rank == 0 or not multi:
        torch.cuda.init()  # torch's HIP runtime first (tests/conftest.py), then libmassrt
        if not multi or world == 1:
            torch.cuda.set_device(0 if multi else (local % torch.cuda.device_count() if world > 1 else 0))
    dev = torch.device("cuda", torch.cuda.current_device())
    solo = n_gpus == 1 and world == 1
    cpu = rank == 0 and solo and not a.no_cpu_baseline

    head = run_scene(a, a.scene, a.steps, a.warmup, rank, world, dev, cpu, devices)
    sec = run_scene(a, secondary, a.secondary_steps, 1, rank, world, dev, cpu, devices) if secondary else None

    dropin, c1, configs = None, None, None
    if rank == 0 and solo and not a.no_dropin:
        dropin = {}
        for sc, ref in ((a.scene, head["value"]), (secondary, sec["value"] if sec else None)):
            if sc:
                try:
                    dropin[sc] = dropin_run(a, sc, ref)
                except Exception as e:
                    dropin[sc] = {"error": str(e)}
    walks = None
    if rank == 0 and solo and not a.no_configs:
        configs = config_lines(a, rank, world, dev, devices)
        walks = other_walk_lines(a, rank, world, dev, devices,
                                 {"headline": head, "secondary": sec, "c3": configs.get("c3")})
    if cpu:
        try:
            c1 = c1_runs(a)
        except Exception as e:
            c1 = {"error": str(e)}

    if rank == 0:
        plan = step_plan(a, n_gpus)
        if multi:
            par = (f"one process, one context over {n_gpus} device(s) {devices} (mrt_create_multi), 8x8 tile "
                   f"shards" + (f" + {head['gather']['transport']} gather onto device 0" if n_gpus > 1 else ""))
        else:
            par = f"tile-shard x{world}" + ((" + RCCL gather" if a.dist_backend == "nccl" else
                                            f" + {a.dist_backend} gather") if world > 1 else "")
        line = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "Msamples/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": plan["scaling"],
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (built-in scene, fixed seeds)",
            "config": {
                "workload": plan["workload"],
                "scene": a.scene, "width": a.width, "height": a.height, "spp_per_step": head["spp_per_step"],
                "samples_per_step": head["samples_per_step"], "max_depth": a.max_depth,
                "parallelism": par, "mode": a.mode,
                "mean_bounces_per_sample": head.get("mean_bounces_per_sample"),
                "mrays_per_s": head.get("mrays_per_s"),
                "scene_load_s": head["scene_load_s"],
                "tuning": head.get("tuning"),
            },
            "roofline": head["roofline"],
            "cpu_baseline": head.get("cpu_baseline"),
        }
        for k, v in head.items():
            if k.startswith("gpu_over_cpu"):
                line["config"][k] = v
        if c1:
            line["config"]["c1"] = c1
        if dropin:
            line["config"]["dropin"] = dropin
        if configs:
            line["config"].update(configs)
        if walks:
            line["config"]["walks"] = walks
        line["config"]["walk"] = WALK_NAMES.get(int((head.get("tuning") or {}).get("traversal", 0)))
        if head.get("roofline_k_shade"):
            line["roofline_k_shade"] = head["roofline_k_shade"]
        if head.get("gather"):
            line["config"]["gather"] = head["gather"]
        tree = src_hash()
        line["build"] = {"library": massrt.build_info(), "tree": f"src {tree}",
                         "match": massrt.build_info() == f"src {tree}"}
        if sec:
            sec["workload"] += " (north_star target: 1M-triangle binary PLY, BASELINE config 4)"
            line["config"]["secondary"] = sec
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
