#!/bin/bash
# Bench A/B over library builds (MASSRT_LIB=<path>.so), no tests: timing only.
#   LIBS="massrt/libmassrt.so massrt/libmassrt_x.so" SCENES="sphere_grid mesh_ply" bash tools/gpu_libab.sh
set -o pipefail
mkdir -p gpurun_out/libab; export TMPDIR=/tmp
for sc in ${SCENES:-sphere_grid}; do
  for lib in $LIBS; do
    tag=$(basename $lib .so)
    MASSRT_LIB=$PWD/mass-raytrace_amd/$lib timeout -k 10 300 python bench.py --scene $sc --secondary none --no-cpu-baseline --steps ${STEPS:-6} > gpurun_out/libab/${sc}_$tag.log 2>&1 || { echo "FAILED $sc $tag"; tail -5 gpurun_out/libab/${sc}_$tag.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/libab/${sc}_$tag.log').read().strip().splitlines()[-1]); r=j['roofline']; print('%-12s %-22s %8.1f  %7.3f ms  util %.3f  exact %.4f' % ('$sc', '$tag', j['value'], r['avg_launch_ms'], r['lane_utilisation'], r.get('box_exact_frac', -1)))"
  done
done
