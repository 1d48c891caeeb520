mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "not mesh" > gpurun_out/quick_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 > gpurun_out/b_def.log 2>&1 && \
MRT_TRACE_WGS_PER_CU=4 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 > gpurun_out/b_4.log 2>&1
rc=$?; echo rc=$rc; tail -2 gpurun_out/quick_tests.log
for f in def 4; do python -c "import json,sys;d=json.loads(open('gpurun_out/b_$f.log').read().strip().splitlines()[-1]);print('$f',d['value'],d['roofline']['avg_launch_ms'],d['roofline']['launches'])"; done
exit $rc
