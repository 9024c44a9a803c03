#!/bin/bash
# Bench part timings (predicted N-GPU efficiency) vs frames in flight (hardware queues = F + 1)
set -o pipefail
OUT=gpurun_out/${1:-parts}
mkdir -p $OUT
for cfg in "160 8" "160 12" "160 16" "160 6"; do
  set -- $cfg
  RTG_BENCH_HW_QUEUES=$(( $2 + 1 )) timeout -k 10 180 python -u bench.py --steps $1 --inflight $2 --no-cpu-baseline --no-sweep > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { tail -20 $OUT/b_$1_$2.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$OUT/b_$1_$2.json').read().strip().splitlines()[-1])
print('steps $1 inflight $2', d['value'], d['ms_per_step'], {k:(v['max_part_ms'],v['predicted_efficiency']) for k,v in d['parts'].items()})" | tee -a $OUT/summary.txt
done
