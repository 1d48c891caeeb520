#!/bin/bash
# Tuning session: GPU parity subset, then bench variants (env A/B) — each step time-limited.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "not mesh_scene" > gpurun_out/quick_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -1 gpurun_out/quick_tests.log
i=0
for v in "${@:-X=1}"; do
  i=$((i+1))
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 $BENCH_ARGS > gpurun_out/tune_$i.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/tune_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/tune_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$v',d['value'],'trace_ms',r['avg_launch_ms'],'launches',r['launches'],'ms/step',d['ms_per_step'])"
done
