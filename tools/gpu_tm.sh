#!/bin/bash
# Tonemapper parity / cost diagnostic, then the full check sequence.  Usage: gpu_tm.sh <tag>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-tm}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python -u tools/diag_tonemap.py > gpurun_out/$tag/diag_tonemap.log 2>&1
rc=$?; echo "diag_tonemap rc=$rc" > gpurun_out/$tag/tm_status.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_check.sh $tag
