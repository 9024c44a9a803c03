#!/bin/bash
# Select-based closest-hit walk step (libws.so, RTG_WALK_SELECT=1) vs the shipped walk: parity,
# headline and C2 / C5
set -o pipefail
OUT=gpurun_out/${1:-ws}
mkdir -p $OUT
LIB=$PWD/advanced-cpu-raytracing_amd/libws.so
RTGPU_LIB=$LIB timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for k in 1 2; do
for v in base ws; do
  if [ $v = ws ]; then export RTGPU_LIB=$LIB; else unset RTGPU_LIB; fi
  timeout -k 10 120 python -u bench.py --steps 100 --no-cpu-baseline --no-sweep --no-extras > $OUT/$v$k.json 2> $OUT/$v$k.err || { tail -5 $OUT/$v$k.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/$v$k.json').read().strip().splitlines()[-1]); c=d['config']
print('$v', d['value'], d['roofline']['kernels_ms'])" | tee -a $OUT/summary.txt
done; done
for v in base ws; do
  if [ $v = ws ]; then export RTGPU_LIB=$LIB; else unset RTGPU_LIB; fi
  timeout -k 10 200 python -u tools/diag_tree.py c5 c2 > $OUT/tree_$v.log 2>&1 || { cat $OUT/tree_$v.log; exit 1; }
  grep -v amdgpu $OUT/tree_$v.log | sed "s/^/$v /" | tee -a $OUT/summary.txt
done
