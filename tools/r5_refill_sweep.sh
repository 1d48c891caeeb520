#!/bin/bash
# trace_refill on the reference walk's big worlds (Menger instanced, mesh_ply solid)
SWEEP=$'base\nr8 MASSRT_OPTIONS=trace_refill=8\nr12 MASSRT_OPTIONS=trace_refill=12\nr16 MASSRT_OPTIONS=trace_refill=16\nr20 MASSRT_OPTIONS=trace_refill=20\nr24 MASSRT_OPTIONS=trace_refill=24' \
SCENES=menger STEPS=1 BENCH_ARGS="--spp-per-step 64" bash tools/gpu_session.sh sweep || exit 1
SWEEP=$'base256\nr16_256 MASSRT_OPTIONS=trace_refill=16' SCENES=menger STEPS=1 BENCH_ARGS="--spp-per-step 256" bash tools/gpu_session.sh sweep || exit 1
SWEEP=$'base\nr16 MASSRT_OPTIONS=trace_refill=16\nr24 MASSRT_OPTIONS=trace_refill=24' SCENES=mesh_ply STEPS=2 bash tools/gpu_session.sh sweep
