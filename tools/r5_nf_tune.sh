#!/bin/bash
# The proven near-first walk's knobs, one at a time (the round-4 rules were
# tuned on the unproven walk): sphere_grid (headline) and cube_field (C3).
SWEEP=$'base\nr32 MASSRT_OPTIONS=trace_refill=32\nr48 MASSRT_OPTIONS=trace_refill=48\nbm20 MASSRT_OPTIONS=trace_box_min=20\nbm32 MASSRT_OPTIONS=trace_box_min=32\nch256 MASSRT_OPTIONS=trace_chunk=256\nch1k MASSRT_OPTIONS=trace_chunk=1024\nnb16 MASSRT_OPTIONS=trace_nf_batch=16\nnb64 MASSRT_OPTIONS=trace_nf_batch=64\nsw8 MASSRT_OPTIONS=shade_waves=8\npb2 MASSRT_OPTIONS=trace_prim_batch=2' \
SCENES="sphere_grid cube_field" STEPS=2 bash tools/gpu_session.sh sweep
