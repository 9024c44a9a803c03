#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-parts}
mkdir -p $OUT
for rev in "" 1; do
RTG_BENCH_PARTS_REVERSED=$rev timeout -k 10 180 python -u bench.py --no-cpu-baseline --no-sweep > $OUT/b_$rev.json 2> $OUT/b_$rev.err || { tail -20 $OUT/b_$rev.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/b_$rev.json').read().strip().splitlines()[-1])
print('rev=$rev', d['steps'], d['value'], d['ms_per_step'], {k:(v['max_part_ms'],v['predicted_efficiency'], v['part_ms']) for k,v in d['parts'].items()})" | tee -a $OUT/summary.txt
done
