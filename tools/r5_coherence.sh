#!/bin/bash
# ABI v9 shading-coherence counters: their GPU test, then the counting step of
# each bench workload (roofline.k_shade.coherence in the line).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5coh
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread -k "coherence or options" \
  > gpurun_out/r5coh/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5coh/pytest.log; exit 1; }
tail -1 gpurun_out/r5coh/pytest.log
for sc in sphere_grid mesh_ply cube_field; do
  timeout -k 10 300 python bench.py --scene $sc --steps 1 --secondary none --no-cpu-baseline --no-dropin --no-configs > gpurun_out/r5coh/b_$sc.log 2>&1 || { echo "bench fail $sc"; tail -5 gpurun_out/r5coh/b_$sc.log; exit 1; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], (j.get('roofline_k_shade') or {}).get('coherence'))" gpurun_out/r5coh/b_$sc.log $sc
done
timeout -k 10 300 python bench.py --scene mesh_obj_textured --width 3840 --height 2160 --spp-per-step 256 --steps 1 --secondary none --no-cpu-baseline --no-dropin --no-configs > gpurun_out/r5coh/b_c5.log 2>&1 || { echo "bench fail c5"; exit 1; }
python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', j['value'], (j.get('roofline_k_shade') or {}).get('coherence'))" gpurun_out/r5coh/b_c5.log
