#!/bin/bash
# GPU tests, smoke, rocprofv3 stats + PMC of both bench scenes (stamped with
# the source hash), then the default bench (which picks those profiles up).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
SCENE=sphere_grid timeout -k 10 900 bash tools/profile.sh > gpurun_out/prof_sg.log 2>&1 && \
SCENE=mesh_ply timeout -k 10 900 bash tools/profile.sh > gpurun_out/prof_mp.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -n 3 gpurun_out/prof_sg.log gpurun_out/prof_mp.log; tail -2 gpurun_out/bench.log
exit $rc
