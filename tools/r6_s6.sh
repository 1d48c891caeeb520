#!/bin/bash
# Round 6: primitive run (k_trace steps the lanes at a primitive alone while
# at least trace_prim_run of them are at one) — A/B of the threshold.
set -o pipefail
export TMPDIR=/tmp
SCENES=mesh_ply STEPS=2 SWEEP="warm MASSRT_OPTIONS=
off MASSRT_OPTIONS=
p24 MASSRT_OPTIONS=trace_prim_run=24
p32 MASSRT_OPTIONS=trace_prim_run=32
p40 MASSRT_OPTIONS=trace_prim_run=40
p48 MASSRT_OPTIONS=trace_prim_run=48" bash tools/gpu_session.sh sweep || exit 1
SCENES="sphere_grid cube_field" STEPS=1 SWEEP="off MASSRT_OPTIONS=
p32 MASSRT_OPTIONS=trace_prim_run=32
p40 MASSRT_OPTIONS=trace_prim_run=40" bash tools/gpu_session.sh sweep || exit 1
