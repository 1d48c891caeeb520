#!/bin/bash
# Round 6: where the cone walk's time goes on mesh_ply — GPU traversal
# counters of both walks and of the zero-margin build, then PMC profiles of
# the NF walk with cones and of the zero-margin build (tools/profile.sh).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/nf_counters.py mesh_ply > gpurun_out/r6_nfc_cone.log 2>&1 || exit 1
cat gpurun_out/r6_nfc_cone.log
MASSRT_LIB=mass-raytrace_amd/massrt/libmassrt_zr.so timeout -k 10 300 python -u tools/nf_counters.py mesh_ply --nf-only \
  > gpurun_out/r6_nfc_zr.log 2>&1 || exit 1
cat gpurun_out/r6_nfc_zr.log
MASSRT_OPTIONS=traversal=1 SCENE=mesh_ply TAG=_nf bash tools/profile.sh > gpurun_out/r6_prof_nf.log 2>&1 || exit 1
tail -30 gpurun_out/r6_prof_nf.log
MASSRT_LIB=mass-raytrace_amd/massrt/libmassrt_zr.so MASSRT_OPTIONS=traversal=1 SCENE=mesh_ply TAG=_zr bash tools/profile.sh \
  > gpurun_out/r6_prof_zr.log 2>&1 || exit 1
tail -30 gpurun_out/r6_prof_zr.log
