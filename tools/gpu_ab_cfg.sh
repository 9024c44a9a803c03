#!/bin/bash
# A/B of an experimental library build on the fused-kernel workloads (C2-C4 bench lines and
# path-tracing throughput), then its GPU parity + path-tracing tests.
# Usage: gpurun -- bash tools/gpu_ab_cfg.sh <tag> <lib.so relative to the package dir>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; lib=$PWD/advanced-cpu-raytracing_amd/$2
out=gpurun_out/$tag
mkdir -p $out
for c in c2 c3 c4; do
  for v in base exp; do
    if [ $v = exp ]; then export RTGPU_LIB=$lib; else unset RTGPU_LIB; fi
    timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_${c}_$v.log 2>&1
    rc=$?; echo "bench $c $v rc=$rc" >> $out/status.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
for v in base exp; do
  if [ $v = exp ]; then export RTGPU_LIB=$lib; else unset RTGPU_LIB; fi
  for s in pt_cornell pt_nee; do
    timeout -k 10 120 python tools/diag_pt.py $s 1024 16 > $out/pt_${s}_$v.log 2>&1
    rc=$?; echo "pt $s $v rc=$rc" >> $out/status.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
export RTGPU_LIB=$lib
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_pathtrace.py -q -x > $out/pytest_exp.log 2>&1
rc=$?; echo "pytest exp rc=$rc" >> $out/status.txt
exit $rc
