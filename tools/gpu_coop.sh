#!/bin/bash
# Cooperative vs sequential large-leaf walks on one configuration (RTG_NO_COOP).
# Usage: gpurun -- bash tools/gpu_coop.sh <tag> <config> [config ...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p $out
for c in "$@"; do
  echo "== $c coop" >> $out/coop.log
  timeout -k 10 300 python tools/diag_config.py $c >> $out/coop.log 2>&1 || exit 1
  echo "== $c seq" >> $out/coop.log
  RTG_NO_COOP=1 timeout -k 10 300 python tools/diag_config.py $c >> $out/coop.log 2>&1 || exit 1
done
