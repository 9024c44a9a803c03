#!/bin/bash
# Headline A/B of library builds, interleaved twice (base, lib1, lib2, ..., base, lib1, ...),
# then the shadow and parity GPU tests on every experimental library.
# Usage: gpurun -- bash tools/gpu_ab_head.sh <tag> <lib.so> [lib.so ...]   (libs relative to the
# package dir; "base" = the default librtgpu.so)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
for rep in 1 2; do
  for l in "$@"; do
    if [ $l = base ]; then unset RTGPU_LIB; else export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l; fi
    timeout -k 10 150 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-sweep --no-extras > $out/bench_${l}_$rep.log 2>&1
    rc=$?; echo "bench $l $rep rc=$rc" >> $st
    [ $rc -ne 0 ] && exit $rc
  done
done
for l in "$@"; do
  [ $l = base ] && continue
  export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l
  timeout -k 10 600 python -u -m pytest tests/test_gpu_shadow.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $out/pytest_$l.log 2>&1
  rc=$?; echo "pytest $l rc=$rc" >> $st
  [ $rc -ne 0 ] && exit $rc
done
exit 0
