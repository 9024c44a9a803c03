#!/bin/bash
# Traversal-variant cost: one configuration's kernel timings with extra feature bits forced
# (RTG_FEAT_FORCE selects a more general kernel; results are unchanged).
# Usage: gpurun -- bash tools/gpu_feat.sh <tag> <config> <bits> [bits ...]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/$1; cfg=$2; shift 2
mkdir -p $out
for b in "$@"; do
  echo "== RTG_FEAT_FORCE=$b" >> $out/feat.log
  RTG_FEAT_FORCE=$b timeout -k 10 300 python tools/diag_config.py $cfg >> $out/feat.log 2>&1 || exit 1
done
