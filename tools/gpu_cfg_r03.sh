#!/bin/bash
# One bench line per configuration (C2-C5, C3 on ton_Roosendaal) + path tracing fused vs wavefront
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-cfg}
mkdir -p $out
for c in c2 c3 c3ton c4 c5; do
  steps=20; [ $c = c5 ] && steps=3; [ $c = c2 ] && steps=100
  timeout -k 10 400 python bench.py --config $c --steps $steps --warmup 1 --no-cpu-baseline > $out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc" >> $out/status.txt
  if [ $rc -ne 0 ]; then tail -20 $out/bench_$c.log; exit $rc; fi
  tail -1 $out/bench_$c.log >> $out/configs.jsonl
done
timeout -k 10 300 python -u tools/diag_ptwave.py 1024 16 > $out/ptwave.log 2>&1 || { cat $out/ptwave.log; exit 1; }
python3 - <<PY
import json
for l in open("$out/configs.jsonl"):
    d = json.loads(l)
    print(d["config"]["workload"][:60], d["value"], d["ms_per_step"], d["roofline"].get("kernels_ms"))
PY
cat $out/ptwave.log
