#!/bin/bash
# Survivor-grouping keys with the LDS-atomic reservation: kind x octant of the
# new ray (library default), kind, octant, kind x (d.y < 0); parity first.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5keys
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread -k "shade_bin or options or coherence" \
  > gpurun_out/r5keys/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5keys/pytest.log; exit 1; }
tail -1 gpurun_out/r5keys/pytest.log
L=mass-raytrace_amd/massrt
SWEEP="kindoct
kind MASSRT_LIB=$L/libmassrt_key0.so
octant MASSRT_LIB=$L/libmassrt_key1.so
kindy MASSRT_LIB=$L/libmassrt_key3.so
nobin MASSRT_OPTIONS=shade_bin=0" SCENES="sphere_grid cube_field mesh_ply" STEPS=2 bash tools/gpu_session.sh sweep
