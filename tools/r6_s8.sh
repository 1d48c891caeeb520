#!/bin/bash
# Round 6: primitive run on by default (trace_prim_run 32) — the frame,
# near-first and parity GPU tests.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_nearfirst.py tests/test_gpu_parity.py tests/test_gpu_benchcall.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_primrun_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r6_primrun_pytest.log
exit $rc
