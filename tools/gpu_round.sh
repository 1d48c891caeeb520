#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the session.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -v -m gpu -x --durations=12 > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
echo "rc=$rc"
tail -22 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -3 gpurun_out/bench.log
exit $rc
