#!/bin/bash
# Kernel trace of C5 on the ray-tree pipeline
set -o pipefail
OUT=gpurun_out/${1:-c5prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-sweep --no-extras > $GRAFT_REPO_ROOT/$OUT/bench.json 2> $GRAFT_REPO_ROOT/$OUT/bench.err || { tail -20 $GRAFT_REPO_ROOT/$OUT/bench.err; exit 1; }
cd $GRAFT_REPO_ROOT
tail -c 600 $OUT/bench.json
