#!/bin/bash
# Round 6: primitive run threshold against the box-run threshold.
set -o pipefail
export TMPDIR=/tmp
SCENES="mesh_ply sphere_grid" STEPS=2 SWEEP="warm MASSRT_OPTIONS=trace_prim_run=32
p16 MASSRT_OPTIONS=trace_prim_run=16
p24 MASSRT_OPTIONS=trace_prim_run=24
p32 MASSRT_OPTIONS=trace_prim_run=32
p32b16 MASSRT_OPTIONS=trace_prim_run=32,trace_box_min=16
p32b24 MASSRT_OPTIONS=trace_prim_run=32,trace_box_min=24
p32b28 MASSRT_OPTIONS=trace_prim_run=32,trace_box_min=28
p24b24 MASSRT_OPTIONS=trace_prim_run=24,trace_box_min=24" bash tools/gpu_session.sh sweep || exit 1
SCENES="cube_field" STEPS=1 SWEEP="p24 MASSRT_OPTIONS=trace_prim_run=24
p32b12 MASSRT_OPTIONS=trace_prim_run=32,trace_box_min=12
p32b20 MASSRT_OPTIONS=trace_prim_run=32,trace_box_min=20" bash tools/gpu_session.sh sweep || exit 1
