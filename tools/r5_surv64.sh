#!/bin/bash
# shade_bin 2 with both survivor counts in one 64-bit atomic per workgroup
# (two 32-bit atomics doubled k_shade's solo time): parity, then shade_bin
# 1 vs 2 on the bench scenes, two queues and solo.
# Measured (profiles/r5_surv64/) with profiles/r5_experiments/surv64.patch
# built as a variant library (MASSRT_LIB=mass-raytrace_amd/massrt/libmassrt_surv64.so,
# make OUT=massrt/libmassrt_surv64.so BUILD=build_surv64); the patch is in
# the source since, so the script now measures the default library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/session
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread -k "shade_bin or options" \
  > gpurun_out/session/pytest_bin.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/session/pytest_bin.log; exit 1; }
tail -1 gpurun_out/session/pytest_bin.log
SWEEP=$'b1 MASSRT_OPTIONS=shade_bin=1\nb2 MASSRT_OPTIONS=shade_bin=2\nsolo_b1 MASSRT_OPTIONS=shade_bin=1,queues=1\nsolo_b2 MASSRT_OPTIONS=shade_bin=2,queues=1' \
  SCENES="sphere_grid cube_field mesh_ply" STEPS=2 bash tools/gpu_session.sh sweep &&
SWEEP=$'b1 MASSRT_OPTIONS=shade_bin=1\nb2 MASSRT_OPTIONS=shade_bin=2' SCENES=mesh_obj_textured STEPS=1 \
  BENCH_ARGS="--width 3840 --height 2160 --spp-per-step 256 --total-spp 256" bash tools/gpu_session.sh sweep
