#!/bin/bash
# Headline: any-hit tree build parameters (RTG_AHB_LEAF, RTG_AHB_CI) and the wide walk's
# occupancy (RTG_WIDE_WAVES_PLAIN builds libw4 / libw6) -- one bench line each
set -o pipefail
OUT=gpurun_out/${1:-ahbtune}
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 100 --no-cpu-baseline --no-sweep --no-extras > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); c=d['config']
print('$name', d['value'], d['roofline']['kernels_ms'], c['shadow_wide_node_visits_per_ray'], c['shadow_tri_tests_per_ray'])" | tee -a $OUT/summary.txt
}
run base RTG_X=0
run leaf1 RTG_AHB_LEAF=1
run leaf4 RTG_AHB_LEAF=4
run leaf8 RTG_AHB_LEAF=8
run ci1 RTG_AHB_CI=1
run ci4 RTG_AHB_CI=4
run ci8 RTG_AHB_CI=8
run w4 RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/libw4.so
run w6 RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/libw6.so
run base2 RTG_X=0
