#!/bin/bash
# A/B of the product library against an experiment library (LIB_B), both on
# the same box: GPU tests of the product first, then bench per scene.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for sc in ${SCENES:-sphere_grid mesh_ply cube_field menger}; do
  for L in "" $LIB_B; do
    log=gpurun_out/ab_${sc}_$(basename "${L:-product}").log
    MASSRT_LIB=$L timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps ${STEPS:-6} > $log 2>&1 || { echo "bench $sc $L failed"; tail -5 $log; exit 1; }
    python3 -c "import json; j=json.loads([l for l in open('$log') if l.startswith('{')][-1]); r=j['roofline']; print('$sc', '$(basename "${L:-product}")', j['value'], r['avg_launch_ms'], r['lane_utilisation'])"
  done
done
