#!/bin/bash
# Quick GPU session: parity subset + division self-test + bench (no CPU baseline)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "not mesh" > gpurun_out/quick_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/quick_bench.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 gpurun_out/quick_tests.log; tail -2 gpurun_out/quick_bench.log
exit $rc
