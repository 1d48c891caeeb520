#!/bin/bash
# What the near-first walk's proof costs on the device (measurement builds):
# zero rounding margins (NOT exact) and a 6-wave occupancy target, with the
# default and a 4 WG/CU grid; then the Menger reference-walk knob sweep.
#   make -C mass-raytrace_amd OUT=massrt/libmassrt_zr.so BUILD=build_zr EXTRA=-DMRT_PROBE_NF_ZERO_RHO massrt/libmassrt_zr.so
#   make -C mass-raytrace_amd OUT=massrt/libmassrt_w6.so BUILD=build_w6 EXTRA=-DMRT_NF_WAVES=6 massrt/libmassrt_w6.so
L=mass-raytrace_amd/massrt
SWEEP="base
c4 MASSRT_OPTIONS=trace_wgs_per_cu=4
zr MASSRT_LIB=$L/libmassrt_zr.so
w6 MASSRT_LIB=$L/libmassrt_w6.so
w6c4 MASSRT_LIB=$L/libmassrt_w6.so MASSRT_OPTIONS=trace_wgs_per_cu=4" \
SCENES="sphere_grid cube_field" STEPS=2 bash tools/gpu_session.sh sweep || exit 1
bash tools/r5_menger_sweep.sh
