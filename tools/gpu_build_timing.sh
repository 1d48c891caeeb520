set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bvh.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bvh.log 2>&1 && \
timeout -k 10 300 python -u tools/build_timing.py > gpurun_out/build_timing.log 2>&1
rc=$?; tail -3 gpurun_out/bvh.log; cat gpurun_out/build_timing.log; exit $rc
