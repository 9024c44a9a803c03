#!/bin/bash
# Bench several in-tree library builds on several configurations (A/B/C... experiments).
# Usage: gpu_libs.sh <tag> "<configs>" lib1.so [lib2.so ...]   (libs relative to the package dir)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; cfgs=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for c in $cfgs; do
  for lib in "$@"; do
    i=$((i+1)); steps=20; [ $c != headline ] && steps=3
    RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/$lib timeout -k 10 300 python bench.py --config $c --steps $steps --warmup 1 --no-cpu-baseline --no-sweep --no-extras > $out/bench_${c}_${i}_${lib%.so}.log 2>&1
    rc=$?; echo "bench $c $lib rc=$rc" >> $out/status.txt
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
