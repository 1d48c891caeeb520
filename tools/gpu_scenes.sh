#!/bin/bash
# Bench the other BASELINE configs' scenes (C3 cube_field, C4 mesh_ply / mesh_obj,
# C5 mesh_obj_textured) at reduced spp per step; each run time-limited.
mkdir -p gpurun_out; export TMPDIR=/tmp
for sc in ${SCENES:-cube_field mesh_ply mesh_obj mesh_obj_textured}; do
  W=1920; H=1080
  if [ "$sc" = "mesh_obj_textured" ]; then W=3840; H=2160; fi
  timeout -k 10 400 python bench.py --no-cpu-baseline --scene $sc --width $W --height $H --steps ${STEPS:-2} --warmup 1 --spp-per-step ${SPP:-16} > gpurun_out/scene_$sc.log 2>&1 || { echo "bench $sc failed"; tail -5 gpurun_out/scene_$sc.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/scene_$sc.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$sc',d['value'],'Msamples/s','trace_ms',r['avg_launch_ms'],'launches',r['launches'],'lane_util',r.get('lane_utilisation'),'bytes/seg',r['bytes_per_segment'],'segs/sample',r['segments_per_sample'])"
done
