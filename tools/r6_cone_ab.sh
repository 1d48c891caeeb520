#!/bin/bash
# Round 6: the near-first walk with per-node normal cones (nf_bound.h
# nf_cone_rg) — parity first (the NF GPU tests, the mesh frames included),
# then mesh_ply on both walks and sphere_grid / cube_field on AUTO.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_nearfirst.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6_cone_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r6_cone_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SWEEP="nf MASSRT_OPTIONS=traversal=1
ref MASSRT_OPTIONS=traversal=0" SCENES="mesh_ply" STEPS=2 bash tools/gpu_session.sh sweep || exit 1
SWEEP="auto MASSRT_OPTIONS=" SCENES="sphere_grid cube_field" STEPS=1 bash tools/gpu_session.sh sweep
