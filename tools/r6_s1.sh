#!/bin/bash
# Round 6, first box of the re-entered session: the GPU suite and smoke on
# the cone source, then mesh_ply on both walks, the per-ray split
# (nf_kappa_log2: camera rays to the reference walk), and the traversal
# counters of both walks.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_session.sh tests || exit 1
SCENES=mesh_ply STEPS=2 SWEEP=$'nf MASSRT_OPTIONS=traversal=1\nref MASSRT_OPTIONS=traversal=0\nk10 MASSRT_OPTIONS=traversal=1,nf_kappa_log2=-10\nk11 MASSRT_OPTIONS=traversal=1,nf_kappa_log2=-11\nzr MASSRT_LIB=mass-raytrace_amd/massrt/libmassrt_zr.so MASSRT_OPTIONS=traversal=1' \
  bash tools/gpu_session.sh sweep || exit 1
timeout -k 10 300 python -u tools/nf_counters.py mesh_ply > gpurun_out/r6_nfc.log 2>&1 || exit 1
cat gpurun_out/r6_nfc.log
