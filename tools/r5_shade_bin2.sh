#!/bin/bash
# shade_bin keys: the material kind (library default) vs the material index's
# low bits (libmassrt_binidx.so); and shade_bin on C5 / Menger.
L=mass-raytrace_amd/massrt
SWEEP="kind MASSRT_OPTIONS=shade_bin=1
idx MASSRT_LIB=$L/libmassrt_binidx.so MASSRT_OPTIONS=shade_bin=1" SCENES="sphere_grid cube_field" STEPS=2 bash tools/gpu_session.sh sweep || exit 1
SWEEP=$'c5bin0 MASSRT_OPTIONS=shade_bin=0\nc5bin1 MASSRT_OPTIONS=shade_bin=1' SCENES=mesh_obj_textured STEPS=2 \
  BENCH_ARGS="--width 3840 --height 2160 --spp-per-step 256" bash tools/gpu_session.sh sweep || exit 1
SWEEP=$'mbin0 MASSRT_OPTIONS=shade_bin=0\nmbin1 MASSRT_OPTIONS=shade_bin=1' SCENES=menger STEPS=1 BENCH_ARGS="--spp-per-step 64" bash tools/gpu_session.sh sweep
