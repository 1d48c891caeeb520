#!/bin/bash
# Option shade_bin (k_shade groups each workgroup's survivors by material
# kind in the next pool): parity tests, then A/B on the bench workloads.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5bin
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread -k "coherence or shade_bin or options" \
  > gpurun_out/r5bin/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5bin/pytest.log; exit 1; }
tail -1 gpurun_out/r5bin/pytest.log
SWEEP=$'bin0 MASSRT_OPTIONS=shade_bin=0\nbin1 MASSRT_OPTIONS=shade_bin=1\nbin0b MASSRT_OPTIONS=shade_bin=0\nbin1b MASSRT_OPTIONS=shade_bin=1' \
SCENES="sphere_grid cube_field mesh_ply" STEPS=2 bash tools/gpu_session.sh sweep
