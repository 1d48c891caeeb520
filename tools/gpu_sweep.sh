#!/bin/bash
# Bench sweep over env configurations: each line of $SWEEP is "label ENV=.. ENV=..";
# scenes in $SCENES. Prints scene, label, Msamples/s, avg k_trace launch ms, lane utilisation.
set -o pipefail
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
SCENES=${SCENES:-"sphere_grid mesh_ply"}
STEPS=${STEPS:-6}
while IFS= read -r line; do
  [ -z "$line" ] && continue
  set -- $line
  label=$1; shift
  for sc in $SCENES; do
    log=gpurun_out/sweep/${sc}_${label}.log
    env "$@" timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps $STEPS > $log 2>&1 || { echo "FAILED $sc $label"; tail -5 $log; exit 1; }
    python3 -c "import json; j=json.loads(open('$log').read().strip().splitlines()[-1]); r=j['roofline']; print('%-12s %-24s %8.1f  %7.3f ms  util %.3f' % ('$sc', '$label', j['value'], r['avg_launch_ms'], r['lane_utilisation']))"
  done
done <<< "$SWEEP"
