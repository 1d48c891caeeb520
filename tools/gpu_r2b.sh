#!/bin/bash
# Treelet session: GPU tests, then a bench sweep of block size / treelet budget.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread --durations=12 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for cfg in "256 0" "1024 78" "1024 150" "512 48" "256 24"; do
  set -- $cfg
  for sc in sphere_grid mesh_ply cube_field; do
    MRT_TRACE_BLOCK=$1 MRT_TREELET_KB=$2 timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps 6 > gpurun_out/sw_${sc}_$1_$2.log 2>&1 || { echo "bench $sc $cfg failed"; tail -5 gpurun_out/sw_${sc}_$1_$2.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/sw_${sc}_$1_$2.log').read().strip().splitlines()[-1]); print('$sc', '$1', '$2', j['value'], j['roofline']['avg_launch_ms'], j['roofline']['lane_utilisation'])"
  done
done
