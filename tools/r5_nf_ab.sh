set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5nf
timeout -k 10 500 python -u -m pytest tests/test_gpu_nearfirst.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5nf/pytest_nf.log 2>&1; echo "pytest rc $?"; tail -3 gpurun_out/r5nf/pytest_nf.log
for sc in sphere_grid mesh_ply cube_field; do
  for tr in 0 1; do
    MASSRT_OPTIONS=traversal=$tr timeout -k 10 300 python bench.py --scene $sc --steps 2 --secondary none --no-cpu-baseline --no-dropin --no-configs > gpurun_out/r5nf/b_${sc}_$tr.log 2>&1 || { echo "bench fail $sc $tr"; tail -3 gpurun_out/r5nf/b_${sc}_$tr.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=j['roofline'] or {}; print(sys.argv[2], sys.argv[3], round(j['value'],1), 'k_trace ms', r.get('avg_launch_ms'))" gpurun_out/r5nf/b_${sc}_$tr.log $sc $tr
  done
done
