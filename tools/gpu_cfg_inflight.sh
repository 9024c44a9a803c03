#!/bin/bash
# Config bench lines with 1 vs 8 frames in flight
set -o pipefail
OUT=gpurun_out/${1:-cfginf}
mkdir -p $OUT
for c in c3 c3ton c4 c2; do
  for f in 1 8; do
    steps=20; [ $c = c2 ] && steps=100
    timeout -k 10 300 python bench.py --config $c --inflight $f --steps $steps --warmup 2 --no-cpu-baseline --no-extras > $OUT/${c}_$f.json 2> $OUT/${c}_$f.err || { tail -5 $OUT/${c}_$f.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/${c}_$f.json').read().strip().splitlines()[-1])
print('$c inflight $f', d['value'], d['ms_per_step'], d['config'].get('serial',{}).get('ms_per_step'))" | tee -a $OUT/summary.txt
  done
done
