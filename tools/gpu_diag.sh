#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-diag}; shift
mkdir -p $out
for c in "$@"; do
  timeout -k 10 300 python tools/diag_config.py $c >> $out/diag.log 2>&1 || exit 1
done
