#!/bin/bash
# Every BASELINE config scene on 1 MI355X (timing only, no CPU baseline), one log line each:
# C2 sphere_grid 1080p, C3 cube_field 1080p, C4 mesh_ply / mesh_obj 1080p, C5 mesh_obj_textured 4K
# (16 spp per step), Menger 20^5 1080p.
set -o pipefail
mkdir -p gpurun_out/configs; export TMPDIR=/tmp
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 600 python bench.py --secondary none --no-cpu-baseline "$@" > gpurun_out/configs/$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 gpurun_out/configs/$tag.log; return 1; }
  python3 -c "import json; j=json.loads(open('gpurun_out/configs/$tag.log').read().strip().splitlines()[-1]); r=j['roofline']; c=j['config']; print('%-22s %-28s %8.1f Msamples/s  %8.1f ms/step  %.2f seg/sample  box_exact %.4f' % ('$tag', c['workload'][:28], j['value'], j['ms_per_step'], r['segments_per_sample'], r['box_exact_frac']))"
}
run c2_sphere_grid --scene sphere_grid --steps 8 && \
run c3_cube_field --scene cube_field --steps 6 && \
run c4_mesh_ply --scene mesh_ply --steps 8 && \
run c4_mesh_obj --scene mesh_obj --steps 8 && \
run c5_mesh_obj_textured_4k --scene mesh_obj_textured --width 3840 --height 2160 --spp-per-step 16 --total-spp 4096 --steps 6 && \
run menger --scene menger --steps 2
