#!/bin/bash
# Round 6: the near-first walk on a mesh scene without the wild light
# instances (mesh_obj_textured: the same 1M-triangle mesh, floor, sky; no
# thin light boxes) — sizes what the never-culled wild instances cost mesh_ply.
set -o pipefail
export TMPDIR=/tmp
SCENES=mesh_obj_textured STEPS=2 SWEEP=$'nf MASSRT_OPTIONS=traversal=1\nref MASSRT_OPTIONS=traversal=0' bash tools/gpu_session.sh sweep || exit 1
timeout -k 10 300 python -u tools/nf_counters.py mesh_obj_textured > gpurun_out/r6_nfc_textured.log 2>&1 || exit 1
cat gpurun_out/r6_nfc_textured.log
