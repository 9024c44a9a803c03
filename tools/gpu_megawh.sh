#!/bin/bash
# Fused kernel ray-tree variants specialised on scene features: parity + C2 timing vs general
set -o pipefail
OUT=gpurun_out/${1:-megawh}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_shadow.py tests/test_gpu_shipped.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/diag_tree.py c2 > $OUT/c2.log 2>&1 || { cat $OUT/c2.log; exit 1; }
RTG_MEGA_GENERAL=1 timeout -k 10 200 python -u tools/diag_tree.py c2 > $OUT/c2_general.log 2>&1 || { cat $OUT/c2_general.log; exit 1; }
grep fused $OUT/c2.log $OUT/c2_general.log
