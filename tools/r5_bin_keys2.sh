#!/bin/bash
# More survivor-grouping keys: kind x (d.y < 0) (key3) vs Lambertian-or-not x
# octant (key4), kind x y-sign x x-sign (key5), y-sign only (key6).
L=mass-raytrace_amd/massrt
SWEEP="kindy MASSRT_LIB=$L/libmassrt_key3.so
lamboct MASSRT_LIB=$L/libmassrt_key4.so
kindyx MASSRT_LIB=$L/libmassrt_key5.so
ysign MASSRT_LIB=$L/libmassrt_key6.so" SCENES="sphere_grid cube_field" STEPS=2 bash tools/gpu_session.sh sweep
