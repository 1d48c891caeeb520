#!/bin/bash
# Round 6: what the proven near-first walk's cost on mesh_ply is made of —
# the margin's VALU (zr: no margin, ncone: the ray's generic term without
# cones), the winner's check (nc), and the grid size (trace_wgs_per_cu) at
# the product and zero-margin register counts (96 / 79 VGPRs).
set -o pipefail
export TMPDIR=/tmp
L=mass-raytrace_amd/massrt
SCENES=mesh_ply STEPS=2 SWEEP="nf MASSRT_OPTIONS=traversal=1
nf_w4 MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=4
nf_w5 MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=5
nf_w2 MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=2
zr_w3 MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=3
zr_w5 MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=5
ncone MASSRT_LIB=$L/libmassrt_ncone.so MASSRT_OPTIONS=traversal=1
nc MASSRT_LIB=$L/libmassrt_nc.so MASSRT_OPTIONS=traversal=1
nf_q1 MASSRT_OPTIONS=traversal=1,queues=1" bash tools/gpu_session.sh sweep
