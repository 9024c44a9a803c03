#!/bin/bash
# GPU parity for C2-C5 at full size + one bench line per configuration.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-cfg}
mkdir -p $out
timeout -k 10 900 python -m pytest tests -q -m gpu -x -s > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $out/status.txt
if [ $rc -gt 1 ]; then exit $rc; fi
for c in c2 c3 c4 c5; do
  timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc" >> $out/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
