#!/bin/bash
# Headline A/B of library builds, interleaved twice (base, lib1, lib2, ..., base, lib1, ...),
# then the shadow and parity GPU tests on every experimental library.
# Usage: gpurun -- bash tools/gpu_ab_head.sh <tag> <lib.so> [lib.so ...]   (libs relative to the
# package dir; "base" = the default librtgpu.so; CONFIGS="headline c3 ..." for other configurations)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
# CONFIGS (environment): the bench configurations to A/B (default: the headline only)
for rep in 1 2; do
  for l in "$@"; do
    if [ $l = base ]; then unset RTGPU_LIB; else export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l; fi
    for c in ${CONFIGS:-headline}; do
      steps=40; [ $c != headline ] && steps=10
      timeout -k 10 200 python bench.py --config $c --steps $steps --warmup 3 --no-cpu-baseline --no-sweep --no-extras > $out/bench_${l}_${c}_$rep.log 2>&1
      rc=$?; echo "bench $l $c $rep rc=$rc" >> $st
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
for l in "$@"; do
  [ $l = base ] && continue
  export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l
  timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_gpu_shadow.py tests/test_gpu_parity.py} -q -x --timeout 300 --timeout-method thread > $out/pytest_$l.log 2>&1
  rc=$?; echo "pytest $l rc=$rc" >> $st
  [ $rc -ne 0 ] && exit $rc
done
exit 0
