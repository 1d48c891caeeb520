timeout -k 10 300 python -u -m pytest tests/test_gpu_nearfirst.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread -k "wild or transport" > gpurun_out/t_wild.log 2>&1; tail -3 gpurun_out/t_wild.log
timeout -k 10 300 python -u tools/nf_counters.py mesh_ply > gpurun_out/nfc.log 2>&1; cat gpurun_out/nfc.log
SCENES=mesh_ply STEPS=2 SWEEP=$'k10 MASSRT_OPTIONS=traversal=1,nf_kappa_log2=-10\nk9 MASSRT_OPTIONS=traversal=1,nf_kappa_log2=-9' bash tools/gpu_session.sh sweep
