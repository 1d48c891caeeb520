#!/bin/bash
# Per-kernel time breakdown with ONE queue (no overlap between the queues'
# kernels, so rocprofv3 durations are isolated) for a few scenes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/breakdown
rm -rf $OUT; mkdir -p $OUT
rc=0
for sc in ${SCENES:-sphere_grid mesh_ply cube_field}; do
  MRT_QUEUES=${QUEUES:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$sc -o run --output-format csv -- python3 bench.py --scene $sc --no-cpu-baseline --steps 4 > $OUT/$sc.log 2>&1 || { rc=$?; echo "$sc failed rc=$rc"; tail -5 $OUT/$sc.log; break; }
  tail -1 $OUT/$sc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc', d['value'], d['roofline']['avg_launch_ms'])"
  f=$(find $OUT/$sc -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):6.2f}")
PY
done
exit $rc
