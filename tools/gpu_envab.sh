#!/bin/bash
# Bench A/B over values of one environment variable (timing only):
#   VAR=MRT_FINISH_PATHS VALS="0 4000000" SCENES="sphere_grid mesh_ply" bash tools/gpu_envab.sh
set -o pipefail
mkdir -p gpurun_out/envab; export TMPDIR=/tmp
for sc in ${SCENES:-sphere_grid}; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps ${STEPS:-6} > gpurun_out/envab/${sc}_$v.log 2>&1 || { echo "FAILED $sc $v"; tail -5 gpurun_out/envab/${sc}_$v.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/envab/${sc}_$v.log').read().strip().splitlines()[-1]); r=j['roofline']; print('%-12s %s=%-10s %8.1f  %7.3f ms/step  trace %7.3f ms  launches %d' % ('$sc', '$VAR', '$v', j['value'], j['ms_per_step'], r['avg_launch_ms'], r['launches']))"
  done
done
