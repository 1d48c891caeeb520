#!/bin/bash
# Is the near-first walk's proof cost instructions or registers? The previous
# build (head, 89 VGPRs), its zero-margin probe (zr, 79; NOT exact) and the
# folded-margin build (fold, 96), each with two queues (traces of both queues
# share the CUs) and with one.
L=mass-raytrace_amd/massrt
SWEEP="head MASSRT_LIB=$L/libmassrt_head.so
zr MASSRT_LIB=$L/libmassrt_zr.so
fold MASSRT_LIB=$L/libmassrt_fold.so
head_q1 MASSRT_LIB=$L/libmassrt_head.so MASSRT_OPTIONS=queues=1
zr_q1 MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=queues=1
fold_q1 MASSRT_LIB=$L/libmassrt_fold.so MASSRT_OPTIONS=queues=1" \
SCENES="sphere_grid" STEPS=2 bash tools/gpu_session.sh sweep
