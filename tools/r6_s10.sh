#!/bin/bash
# Round 6: the reference walk's drop in the bench line's other-walk legs —
# the pre-primitive-run library (libmassrt_old.so, commit 3647faf) against
# the current one, reference walk (traversal=0) and near-first.
set -o pipefail
export TMPDIR=/tmp
L=mass-raytrace_amd/massrt
SCENES="sphere_grid" STEPS=1 SWEEP="warm MASSRT_OPTIONS=traversal=0
t0new MASSRT_OPTIONS=traversal=0
t0old MASSRT_LIB=$L/libmassrt_old.so MASSRT_OPTIONS=traversal=0
t0p65 MASSRT_OPTIONS=traversal=0,trace_prim_run=65
t0new2 MASSRT_OPTIONS=traversal=0
t0old2 MASSRT_LIB=$L/libmassrt_old.so MASSRT_OPTIONS=traversal=0
t1new MASSRT_OPTIONS=traversal=1
t1old MASSRT_LIB=$L/libmassrt_old.so MASSRT_OPTIONS=traversal=1" bash tools/gpu_session.sh sweep || exit 1
