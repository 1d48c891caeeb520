#!/bin/bash
# Round-5 A/B of the walks on the bench scenes: the reference walk, the proven
# near-first walk; one bench line each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/walk_ab
L=mass-raytrace_amd/massrt
one() {  # label scene lib opts extra...
  local lab=$1 sc=$2 lib=$3 opts=$4; shift 4
  MASSRT_LIB=$lib MASSRT_OPTIONS=$opts timeout -k 10 400 python bench.py --scene $sc --secondary none --no-cpu-baseline \
    --no-dropin --no-configs "$@" > gpurun_out/walk_ab/${lab}_$sc.log 2>&1 || { echo "FAILED $lab $sc"; tail -3 gpurun_out/walk_ab/${lab}_$sc.log; return 1; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=j['roofline'] or {}; print('%-8s %-12s %8.1f Msamples/s  k_trace %.2f ms' % (sys.argv[2], sys.argv[3], j['value'], r.get('avg_launch_ms', 0)))" gpurun_out/walk_ab/${lab}_$sc.log $lab $sc
}
for sc in ${SCENES:-sphere_grid cube_field mesh_ply}; do
  one ref $sc $L/libmassrt.so traversal=0 --steps 2 &&
  one nf $sc $L/libmassrt.so traversal=1 --steps 2 || exit 1
done
if [ -n "$MENGER" ]; then
  one ref menger $L/libmassrt.so traversal=0 --steps 1 --spp-per-step 64 &&
  one nf menger $L/libmassrt.so traversal=1 --steps 1 --spp-per-step 64 &&
  one nf64 menger $L/libmassrt.so traversal=1,trace_nf_batch=64 --steps 1 --spp-per-step 64
fi
