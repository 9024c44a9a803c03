#!/bin/bash
# Any-hit tree variants on the fixture scenes and BASELINE configs (tools/diag_ahb.py).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-ahb2}
mkdir -p $out
timeout -k 10 600 python -u tools/diag_ahb.py > $out/diag_ahb.log 2>&1
echo "diag_ahb rc=$?" > $out/status.txt
