#!/bin/bash
# A/B of experiment builds on three scenes: tools/gpu_ab3.sh <lib.so> [<lib.so> ...]
set -o pipefail
args=("X=1")
for l in "$@"; do args+=("MASSRT_LIB=$l"); done
for sc in sphere_grid cube_field mesh_ply; do
  BENCH_ARGS="--scene $sc" bash tools/gpu_ab.sh "${args[@]}" || exit 1
done
