#!/bin/bash
# A/B of an experimental in-tree library build against the default one: headline bench
# with each, then the GPU parity tests on the experimental build.
# Usage: gpurun -- bash tools/gpu_ab.sh <tag> <lib.so relative to the package dir> [bench args]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; lib=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $out/bench_base.log 2>&1
rc=$?; echo "bench base rc=$rc" > $out/status.txt
[ $rc -ne 0 ] && exit $rc
RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $out/bench_exp.log 2>&1
rc=$?; echo "bench exp rc=$rc" >> $out/status.txt
[ $rc -ne 0 ] && exit $rc
RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$lib timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x > $out/pytest_exp.log 2>&1
rc=$?; echo "pytest exp rc=$rc" >> $out/status.txt
exit $rc
