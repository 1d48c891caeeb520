#!/bin/bash
# A/B session: GPU parity tests (all of tests/test_gpu_parity.py except the
# 1M-triangle and Menger scenes unless FULL=1), then one short bench per
# "ENV=VAL ..." argument (default: the default config), each time-limited.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
K="not mesh_scene and not menger"; [ "$FULL" = 1 ] && K=""
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x -k "$K" --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
i=0
for v in "${@:-X=1}"; do
  i=$((i+1))
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-8} $BENCH_ARGS > gpurun_out/ab_$i.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$v',d['config']['scene'],d['value'],'trace_ms',r['avg_launch_ms'],'launches',r['launches'],'util',r['lane_utilisation'])"
done
