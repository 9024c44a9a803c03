#!/bin/bash
# The whole GPU test suite on an experimental library build, then per-configuration bench lines
# for the default and the experimental build.
# Usage: gpurun -- bash tools/gpu_lib_check.sh <tag> <lib.so> "<configs>"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; lib=$2; cfgs=$3
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $st
[ $rc -ne 0 ] && exit $rc
for c in $cfgs; do
  for l in $lib base; do
    if [ $l = base ]; then unset RTGPU_LIB; else export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l; fi
    timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $out/bench_${c}_$l.log 2>&1
    rc=$?; echo "bench $c $l rc=$rc" >> $st
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
