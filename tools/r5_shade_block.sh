#!/bin/bash
# Grouping scope of the survivor grouping (option shade_bin): k_shade's
# workgroup size 256 (default) / 512 / 1024 (libraries built with
# MRT_SHADE_BLOCK: make OUT=massrt/libmassrt_sb<N>.so BUILD=build_sb<N>
# EXTRA=-DMRT_SHADE_BLOCK=<N>), and shade_bin 2 (the y-sign halves at the
# pool's two ends: a pool-wide split). Parity first, then the A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/session
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread -k "shade_bin or options" \
  > gpurun_out/session/pytest_bin.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/session/pytest_bin.log; exit 1; }
tail -1 gpurun_out/session/pytest_bin.log
L=mass-raytrace_amd/massrt
SWEEP="b1 MASSRT_OPTIONS=shade_bin=1
b2 MASSRT_OPTIONS=shade_bin=2
sb1024_b1 MASSRT_LIB=$L/libmassrt_sb1024.so MASSRT_OPTIONS=shade_bin=1
sb1024_b2 MASSRT_LIB=$L/libmassrt_sb1024.so MASSRT_OPTIONS=shade_bin=2
sb512_b1 MASSRT_LIB=$L/libmassrt_sb512.so MASSRT_OPTIONS=shade_bin=1
b1r MASSRT_OPTIONS=shade_bin=1" \
SCENES="sphere_grid cube_field mesh_ply" STEPS=2 bash tools/gpu_session.sh sweep
