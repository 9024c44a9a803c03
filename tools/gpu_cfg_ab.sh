#!/bin/bash
# Per-configuration A/B of library builds, interleaved twice (bench lines with --no-extras).
# Usage: gpurun -- bash tools/gpu_cfg_ab.sh <tag> "<configs>" <lib.so|base> [...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; cfgs=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
for rep in 1 2; do
  for c in $cfgs; do
    for l in "$@"; do
      if [ $l = base ]; then unset RTGPU_LIB; else export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l; fi
      steps=10; [ $c = c5 ] && steps=2
      timeout -k 10 200 python bench.py --config $c --steps $steps --warmup 1 --no-cpu-baseline --no-extras > $out/bench_${c}_${l}_$rep.log 2>&1
      rc=$?; echo "bench $c $l $rep rc=$rc" >> $st
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
