#!/bin/bash
# Round 6: wild instances culled by their own box and margin (nf_bound.h
# NfWild) — the near-first parity tests, then mesh_ply on both walks, the
# zero-margin probe, the headline scenes on AUTO, and the traversal counters.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nearfirst.py tests/test_gpu_benchcall.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6_wild_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r6_wild_pytest.log
[ $rc -eq 0 ] || exit $rc
L=mass-raytrace_amd/massrt
SCENES=mesh_ply STEPS=2 SWEEP="nf MASSRT_OPTIONS=traversal=1
ref MASSRT_OPTIONS=traversal=0
zr MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1" bash tools/gpu_session.sh sweep || exit 1
SCENES="sphere_grid cube_field" STEPS=1 SWEEP="auto MASSRT_OPTIONS=" bash tools/gpu_session.sh sweep || exit 1
timeout -k 10 300 python -u tools/nf_counters.py mesh_ply > gpurun_out/r6_nfc_wild.log 2>&1 || exit 1
cat gpurun_out/r6_nfc_wild.log
