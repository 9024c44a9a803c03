#!/bin/bash
# Parity tests + headline bench + C3 rows diag.  Usage: gpu_quick.sh <tag>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-q}
mkdir -p $out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $out/status.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $out/status.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_rows.py > $out/rows.log 2>&1
echo "rows rc=$?" >> $out/status.txt
