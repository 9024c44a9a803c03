#!/bin/bash
# Quick GPU round: all GPU tests, then the headline bench (no CPU baseline / sweep) and the
# C3 / C4 config lines.  Usage: gpurun --timeout 1200 -- bash tools/gpu_fast.sh <tag> [pytest -k expr]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-fast}
mkdir -p $out
st=$out/status.txt
if [ -n "$2" ]; then k=(-k "$2"); else k=(); fi
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread "${k[@]}" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
for c in c3 c4 c3ton; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-sweep --no-extras > $out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $st
