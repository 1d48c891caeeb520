#!/bin/bash
# Menger on the reference's walk: the trace knobs one at a time (64 spp per run)
SWEEP=$'base\nr16 MASSRT_OPTIONS=trace_refill=16\nr56 MASSRT_OPTIONS=trace_refill=56\nbm8 MASSRT_OPTIONS=trace_box_min=8\nbm48 MASSRT_OPTIONS=trace_box_min=48\nch2k MASSRT_OPTIONS=trace_chunk=2048\nch128 MASSRT_OPTIONS=trace_chunk=128\nq1 MASSRT_OPTIONS=queues=1\npb4 MASSRT_OPTIONS=trace_prim_batch=4\nwg4 MASSRT_OPTIONS=trace_wgs_per_cu=4\nwg8 MASSRT_OPTIONS=trace_wgs_per_cu=8' \
SCENES=menger STEPS=1 BENCH_ARGS="--spp-per-step 64" exec bash tools/gpu_session.sh sweep
