#!/bin/bash
# Kernel trace of the wavefront path tracer (pt_cornell, pt_rr at 1024^2 x 16 spp)
set -o pipefail
OUT=gpurun_out/${1:-ptprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for s in pt_cornell pt_rr; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/$s -o run -- python3 -u $GRAFT_REPO_ROOT/tools/diag_ptwave.py 1024 16 $s > $GRAFT_REPO_ROOT/$OUT/$s.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/$s.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for s in pt_cornell pt_rr; do
  f=$(find $OUT/$s -name "*kernel_stats.csv" | head -1); echo "== $s"; cut -d, -f1-8 $f | head -14
done
