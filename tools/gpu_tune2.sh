#!/bin/bash
# Sweep of the persistent loop's refill threshold and box-run threshold.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
# CONFIGS: comma-separated "refill box_min" pairs
IFS=, read -ra CFGS <<< "${CONFIGS:-32 24,16 24,24 24,16 16,16 32,24 32,32 32,8 24,48 24}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  for sc in ${SCENES:-sphere_grid mesh_ply}; do
    log=gpurun_out/tn_${sc}_$1_$2.log
    MRT_TRACE_REFILL=$1 MRT_TRACE_BOX_MIN=$2 timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps 6 > $log 2>&1 || { echo "bench $sc $cfg failed"; tail -5 $log; exit 1; }
    python3 -c "import json; j=json.loads([l for l in open('$log') if l.startswith('{')][-1]); r=j['roofline']; print('$sc', 'refill', '$1', 'box_min', '$2', j['value'], r['avg_launch_ms'], r['lane_utilisation'])"
  done
done
