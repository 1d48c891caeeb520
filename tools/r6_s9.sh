#!/bin/bash
# Round 6: box-run threshold beside the primitive run (default 32), near-first scenes.
set -o pipefail
export TMPDIR=/tmp
SCENES="mesh_ply sphere_grid" STEPS=2 SWEEP="warm MASSRT_OPTIONS=
b20 MASSRT_OPTIONS=
b16 MASSRT_OPTIONS=trace_box_min=16
b18 MASSRT_OPTIONS=trace_box_min=18
b12 MASSRT_OPTIONS=trace_box_min=12
b20r MASSRT_OPTIONS=
b16r MASSRT_OPTIONS=trace_box_min=16
p28 MASSRT_OPTIONS=trace_prim_run=28
p36 MASSRT_OPTIONS=trace_prim_run=36" bash tools/gpu_session.sh sweep || exit 1
