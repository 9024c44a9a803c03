#!/bin/bash
# Tonemapper log-sum mode 3 (summarised windows): parity tests + cost vs mode 2 / 1
set -o pipefail
OUT=gpurun_out/${1:-tm3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tonemap.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for m in 3 2 1; do
  RTG_TM_SEQSUM=$m timeout -k 10 200 python -u tools/diag_tonemap.py > $OUT/diag_m$m.log 2>&1 || { tail -20 $OUT/diag_m$m.log; exit 1; }
  grep -E "mode|tonemap |golden 0|fullhd" $OUT/diag_m$m.log
done
