#!/bin/bash
# Fused path-tracing kernel: feature-specialised variants vs the general one (RTG_MEGA_GENERAL)
set -o pipefail
OUT=gpurun_out/${1:-megapt}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pathtrace.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/diag_ptwave.py 1024 16 > $OUT/ptwave.log 2>&1 || { cat $OUT/ptwave.log; exit 1; }
RTG_MEGA_GENERAL=1 timeout -k 10 300 python -u tools/diag_ptwave.py 1024 16 > $OUT/ptwave_general.log 2>&1 || { cat $OUT/ptwave_general.log; exit 1; }
grep fused $OUT/ptwave.log; grep fused $OUT/ptwave_general.log
