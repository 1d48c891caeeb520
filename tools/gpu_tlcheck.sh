#!/bin/bash
# Treelet vs plain k_trace at scale: diagnostics, then the full-size parity test.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/treelet_check.py sphere_grid 1024 78 > gpurun_out/tlcheck.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tlcheck.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -m gpu -x -k treelet --timeout 200 --timeout-method thread > gpurun_out/pytest_tl_full.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tl_full.log; exit $rc
