#!/bin/bash
# A/B/C of library builds: one bench line per (config, library), then the GPU parity tests on
# every experimental library.  Usage:
#   gpurun -- bash tools/gpu_ab_multi.sh <tag> "<configs>" <lib.so> [lib.so ...]
# (libs relative to the package dir; "base" = the default librtgpu.so; configs from bench.py)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; cfgs=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for c in $cfgs; do
  for l in "$@"; do
    if [ $l = base ]; then unset RTGPU_LIB; else export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l; fi
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${c}_$l.log 2>&1
    rc=$?; echo "bench $c $l rc=$rc" >> $out/status.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
for l in "$@"; do
  [ $l = base ] && continue
  export RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$l
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_pathtrace.py tests/test_gpu_configs.py -q -x > $out/pytest_$l.log 2>&1
  rc=$?; echo "pytest $l rc=$rc" >> $out/status.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
