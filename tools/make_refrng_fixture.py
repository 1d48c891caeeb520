"""Fixture for the statistical reference-semantics check (SURVEY §4 item 6,
tests/test_gpu_statistical.py): the oracle rendering with the REFERENCE's
RNG semantics (orc_render_refrng: one fastrand wyrand stream per render
worker, consumed in the pixel-loop order of main.rs:253-264 by every draw:
jitter, Camera::ray's disk, scatter, volume/alpha draws; math.rs:244-246,
world.rs:53-63) — 64 workers x 64 passes = 4096 samples of each pixel of a
64x36 frame. Stored per pixel: the radiance mean and per-sample variance
(float32), the bounce-count mean and variance, and the sample count.

The GPU draws from per-(pixel, sample) xoroshiro streams instead:
the two images must agree in distribution, which the test checks block by
block. Run here (CPU, ~1 min):  python tools/make_refrng_fixture.py
"""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mass-raytrace_amd")]

import massrt  # noqa: E402
import oracle  # noqa: E402  (test infrastructure)

W, H, WORKERS, PASSES, SEED = 64, 36, 64, 64, 1


def main():
    for scene in ("cornell", "sphere_grid"):
        t = time.time()
        o = oracle.Scene(1).builtin(scene, float(massrt.ASPECT_RATIO), str(REPO / "tests" / "golden"))
        s, q, b, bq = o.render_refrng(W, H, PASSES, WORKERS, seed=SEED, threads=0)
        n = WORKERS * PASSES
        mean = s / n
        var = np.maximum(q / n - mean * mean, 0.0) * n / (n - 1)
        bmean = b / n
        bvar = np.maximum(bq / n - bmean * bmean, 0.0) * n / (n - 1)
        out = REPO / "tests" / "golden" / f"refrng_{scene}.npz"
        np.savez_compressed(out, mean=mean.astype(np.float32), var=var.astype(np.float32),
                            bmean=bmean.astype(np.float32), bvar=bvar.astype(np.float32), n=np.int64(n),
                            width=W, height=H)
        print(f"{scene}: {n} spp x {W}x{H} in {time.time() - t:.1f}s -> {out.relative_to(REPO)}")


if __name__ == "__main__":
    main()
