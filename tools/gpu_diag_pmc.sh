#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-dpmc}; cfg=$2; shift; shift
mkdir -p $out
k=0
for pass in "$@"; do
  k=$((k+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-include-regex "rtg::k_" -f csv -d $GRAFT_REPO_ROOT/$out/pass$k -o run -- python $cfg > $out/pass$k.log 2>&1 || exit 1
done
