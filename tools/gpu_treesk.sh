#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-treesk}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "tree or c5" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python -u tools/diag_tree.py c5 c2 > $OUT/diag_tree.log 2>&1 || { cat $OUT/diag_tree.log; exit 1; }
cat $OUT/diag_tree.log
