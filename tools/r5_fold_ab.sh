#!/bin/bash
# The near-first walk with its margin folded into the ray (no per-node rho,
# no exit tracking) and the world-ray stash: GPU parity, then A/B against
# the previous build (libmassrt_head.so) on the near-first scenes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5fold
timeout -k 10 600 python -u -m pytest tests/test_gpu_nearfirst.py tests/test_gpu_benchcall.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5fold/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5fold/pytest.log; exit 1; }
tail -2 gpurun_out/r5fold/pytest.log
L=mass-raytrace_amd/massrt
SWEEP="head MASSRT_LIB=$L/libmassrt_head.so
fold" SCENES="sphere_grid cube_field" STEPS=2 bash tools/gpu_session.sh sweep
