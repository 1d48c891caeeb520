#!/bin/bash
# Round-5 stamped PMC profiles of the final source, for every workload of the
# default bench line (the walk each takes under AUTO is stamped and tagged by
# tools/pmc_summary.py): headline sphere_grid (near-first) and its solo run,
# mesh_ply (reference walk) and solo, C3 cube_field (near-first), C5 4K.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/session
p() { echo "profile $*"; env "$@" bash tools/profile.sh > gpurun_out/session/profile_$(echo "$*" | tr ' =/' '___').log 2>&1 || { echo "FAILED $*"; exit 1; }; }
p SCENE=sphere_grid && p SCENE=sphere_grid TAG=_solo MASSRT_OPTIONS=queues=1 && \
p SCENE=mesh_ply && p SCENE=mesh_ply TAG=_solo MASSRT_OPTIONS=queues=1 && \
p SCENE=cube_field && \
p SCENE=mesh_obj_textured BENCH_EXTRA="--width 3840 --height 2160 --spp-per-step 256"
