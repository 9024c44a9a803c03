#!/bin/bash
# 8-row bands: partition tests (multi-GPU composition, parity with parts) + bench part timings
set -o pipefail
OUT=gpurun_out/${1:-parts}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multigpu.py tests/test_gpu_parity.py tests/test_gpu_pathtrace.py -k "part or band or multi or gather or compose or wavefront" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 180 python -u bench.py --steps 160 --no-cpu-baseline --no-sweep > $OUT/b160.json 2> $OUT/b160.err || { tail -20 $OUT/b160.err; exit 1; }
timeout -k 10 180 python -u bench.py --no-cpu-baseline --no-sweep > $OUT/b20.json 2> $OUT/b20.err || { tail -20 $OUT/b20.err; exit 1; }
for f in b160 b20; do python3 -c "
import json
d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1])
print('$f', d['steps'], d['value'], d['ms_per_step'], {k:(v['max_part_ms'],v['predicted_efficiency'], v['part_ms']) for k,v in d['parts'].items()})" | tee -a $OUT/summary.txt; done
