#!/bin/bash
# Tree pipeline with the exact any-hit shadow walk: shadow / tree / C5 parity + C2, C5 timings
set -o pipefail
OUT=gpurun_out/${1:-treesh}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shadow.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "shadow or tree or c5 or C5 or dielectric or mirror" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python -u tools/diag_tree.py c2 c5 > $OUT/diag_tree.log 2>&1 || { cat $OUT/diag_tree.log; exit 1; }
cat $OUT/diag_tree.log
