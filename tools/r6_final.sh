#!/bin/bash
# Round-6 evidence on the final source, in parts that fit one call:
#   bash tools/r6_final.sh 1   # GPU suite + smoke, stamped profiles of the headline (and solo)
#   bash tools/r6_final.sh 2   # stamped profiles of mesh_ply (and solo), C3, C5
#   bash tools/r6_final.sh all # 1, 2 and the bench line in one call
#   bash tools/r6_final.sh 3   # the default bench line, the 2-device rehearsal, shade_bin 1 vs 2 on C5 and Menger,
#                              # the near-first loop knobs re-checked under the split pool
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/session
p() { echo "profile $*"; env "$@" bash tools/profile.sh > gpurun_out/session/profile_$(echo "$*" | tr ' =/' '___').log 2>&1 || { echo "FAILED $*"; tail -20 gpurun_out/session/profile_$(echo "$*" | tr ' =/' '___').log; exit 1; }; }
case $1 in
  1) bash tools/gpu_session.sh tests && p SCENE=sphere_grid && p SCENE=sphere_grid TAG=_solo MASSRT_OPTIONS=queues=1 ;;
  2) p SCENE=mesh_ply && p SCENE=mesh_ply TAG=_solo MASSRT_OPTIONS=queues=1 && p SCENE=cube_field && \
     p SCENE=mesh_obj_textured BENCH_EXTRA="--width 3840 --height 2160 --spp-per-step 256" ;;
  all) bash $0 1 && bash $0 2 && bash tools/gpu_session.sh bench ;;  # one call: suite, smoke, profiles, bench
  3) bash tools/gpu_session.sh bench && bash tools/gpu_session.sh rehearse && \
     SWEEP=$'b1 MASSRT_OPTIONS=shade_bin=1\nb2 MASSRT_OPTIONS=shade_bin=2' SCENES=mesh_obj_textured STEPS=1 \
       BENCH_ARGS="--width 3840 --height 2160 --spp-per-step 256 --total-spp 256" bash tools/gpu_session.sh sweep && \
     SWEEP=$'b1 MASSRT_OPTIONS=shade_bin=1\nb2 MASSRT_OPTIONS=shade_bin=2' SCENES=menger STEPS=1 \
       BENCH_ARGS="--spp-per-step 64" bash tools/gpu_session.sh sweep && \
     SWEEP=$'base\nrf32 MASSRT_OPTIONS=trace_refill=32\nrf48 MASSRT_OPTIONS=trace_refill=48\nch256 MASSRT_OPTIONS=trace_chunk=256\nch1024 MASSRT_OPTIONS=trace_chunk=1024\nbm20 MASSRT_OPTIONS=trace_box_min=20\nbm28 MASSRT_OPTIONS=trace_box_min=28' \
       SCENES="sphere_grid cube_field" STEPS=2 bash tools/gpu_session.sh sweep ;;
esac
