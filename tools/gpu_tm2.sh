#!/bin/bash
# Tonemapper GPU tests + diagnostics for the windowed (2) and chained (1) log-sum.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-tm2}
mkdir -p $out
st=$out/status.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_tonemap.py -v -s -m gpu -x --timeout 200 --timeout-method thread > $out/pytest_tm.log 2>&1
rc=$?; echo "pytest tonemap rc=$rc" > $st
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 2 1; do
  RTG_TM_SEQSUM=$m timeout -k 10 300 python -u tools/diag_tonemap.py > $out/diag_tonemap_m$m.log 2>&1
  rc=$?; echo "diag_tonemap m$m rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
done
