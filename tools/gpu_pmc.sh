#!/bin/bash
# One rocprofv3 --pmc pass per argument (quoted counter lists) over a short bench.
# Usage: gpu_pmc.sh <tag> "<counters pass 1>" ["<counters pass 2>" ...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
k=0
for pass in "$@"; do
  k=$((k+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-include-regex "rtg::k_" -f csv -d $out/pass$k -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/pass$k.log 2>&1
  rc=$?; echo "pass$k ($pass) rc=$rc" >> $out/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
