#!/bin/bash
# GPU tests + smoke, then the evidence run (rocprofv3 stats + stamped PMC for
# both bench scenes, then the default bench line). Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread --durations=8 > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu_evidence.sh
