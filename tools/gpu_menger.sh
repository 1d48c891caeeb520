#!/bin/bash
# Menger on the GPU: parity tests, then benches of menger and mesh_ply.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -x -k menger --timeout 300 --timeout-method thread > gpurun_out/menger_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --scene menger --steps 4 > gpurun_out/bench_menger.log 2>&1 && \
timeout -k 10 300 python bench.py --scene mesh_ply --steps 8 > gpurun_out/bench_mesh_ply.log 2>&1
rc=$?
echo "rc=$rc"; tail -8 gpurun_out/menger_tests.log; tail -1 gpurun_out/bench_menger.log; tail -1 gpurun_out/bench_mesh_ply.log
exit $rc
