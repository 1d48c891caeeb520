#!/bin/bash
# Round 6: why the proven near-first walk is slow on mesh_ply (1M generic
# triangles): measurement builds without the rounding margin (zr), without
# the winner's check (nc), both (zrnc), and the NF grid at 4/5 WG per CU.
#   make -C mass-raytrace_amd OUT=massrt/libmassrt_zr.so BUILD=build_zr EXTRA=-DMRT_PROBE_NF_ZERO_RHO massrt/libmassrt_zr.so
#   make -C mass-raytrace_amd OUT=massrt/libmassrt_nc.so BUILD=build_nc EXTRA=-DMRT_PROBE_NF_NOCHECK massrt/libmassrt_nc.so
L=mass-raytrace_amd/massrt
SWEEP="nf MASSRT_OPTIONS=traversal=1
zr MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1
nc MASSRT_LIB=$L/libmassrt_nc.so MASSRT_OPTIONS=traversal=1
zrnc MASSRT_LIB=$L/libmassrt_zrnc.so MASSRT_OPTIONS=traversal=1
c5 MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=5
c4 MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=4
zrc5 MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1,trace_wgs_per_cu=5" \
SCENES="mesh_ply" STEPS=1 bash tools/gpu_session.sh sweep
