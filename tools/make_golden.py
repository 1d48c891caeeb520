"""Generate tests/golden/oracle_golden.npz: small fixed-seed renders and ray
batches produced by the oracle (oracle/oracle.cpp). They pin the oracle across
rounds (any change to its arithmetic shows up as a fixture diff) and are the
committed vectors the GPU parity tests also compare against.

Provenance: the reference cannot be built or run here (no Rust toolchain, 215
crates absent), so these are restatement outputs, not reference outputs.
Usage: python tools/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "mass-raytrace_amd"))

import oracle  # noqa: E402

ASPECT = float(np.float32(16.0) / np.float32(9.0))
SCENES = ["cornell", "sphere_grid", "cube_field"]
W, H, SPP, SEED = 32, 18, 2, 3


def golden_rays(n=512, seed=11):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-15, 15, (n, 3)).astype(np.float32)
    o[:, 1] = np.abs(o[:, 1]) + 0.5
    d = rng.normal(size=(n, 3)).astype(np.float32)
    return np.concatenate([o, d], 1)


def main():
    gd = REPO / "tests" / "golden"
    out = {"rays": golden_rays()}
    for s in SCENES:
        sc = oracle.Scene(1).builtin(s, ASPECT, gd)
        rgb, b = sc.render(W, H, 0, SPP, seed=SEED, threads=4)
        out[f"{s}_rgb"] = rgb
        out[f"{s}_bounces"] = b
        out[f"{s}_hits"] = sc.trace_rays(out["rays"])
        out[f"{s}_counters"] = np.array([sc.counters()[k] for k in oracle.COUNTER_FIELDS], dtype=np.uint64)
    np.savez_compressed(gd / "oracle_golden.npz", **out)
    print("wrote", gd / "oracle_golden.npz", sorted(out))


if __name__ == "__main__":
    main()
