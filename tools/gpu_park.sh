#!/bin/bash
# Treelet with parked global loads: full-size parity (product lib, then the
# experiment libs named in LIBS), the treelet budget tests, then a sweep of
# workgroup size / treelet budget / box-run threshold.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in "" ${LIBS}; do
  timeout -k 10 300 env MASSRT_LIB=$L python -u -m pytest tests/test_gpu_fullsize.py -v -m gpu -x -k "treelet" --timeout 200 --timeout-method thread > gpurun_out/pytest_park_full$(basename "$L").log 2>&1
  echo "fullsize lib=${L:-product} rc=$?"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -m gpu -x -k "treelet" --timeout 200 --timeout-method thread > /dev/null 2>&1 || { echo "product fullsize parity fails: no sweep"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -x -k "treelet or model_blas or golden" --timeout 300 --timeout-method thread > gpurun_out/pytest_park.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_park.log
[ $rc -ne 0 ] && exit $rc
for cfg in ${CONFIGS:-"256 0 24" "1024 78 24" "512 48 24" "256 24 24" "1024 78 16" "1024 78 32"}; do
  set -- $cfg
  for sc in ${SCENES:-sphere_grid mesh_ply cube_field}; do
    log=gpurun_out/pk_${sc}_$1_$2_$3.log
    MRT_TRACE_BLOCK=$1 MRT_TREELET_KB=$2 MRT_TRACE_BOX_MIN=$3 timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps 6 > $log 2>&1 || { echo "bench $sc $cfg failed"; tail -5 $log; exit 1; }
    python3 -c "import json; j=json.loads([l for l in open('$log') if l.startswith('{')][-1]); r=j['roofline']; print('$sc', '$1', '$2', '$3', j['value'], r['avg_launch_ms'], r['lane_utilisation'])"
  done
done
