#!/bin/bash
# k_shade workgroup size (the scope of the shade_bin survivor grouping):
# 256 (default) vs 512 vs 1024 threads, libraries built with
# MRT_SHADE_BLOCK (make OUT=massrt/libmassrt_sb<N>.so BUILD=build_sb<N> EXTRA=-DMRT_SHADE_BLOCK=<N>).
set -o pipefail
export TMPDIR=/tmp
LABELS="sb256 sb512 sb1024 sb256b" \
LIBS="mass-raytrace_amd/massrt/libmassrt.so mass-raytrace_amd/massrt/libmassrt_sb512.so mass-raytrace_amd/massrt/libmassrt_sb1024.so mass-raytrace_amd/massrt/libmassrt.so" \
SCENES="sphere_grid cube_field mesh_ply" STEPS=2 bash tools/gpu_session.sh ab
