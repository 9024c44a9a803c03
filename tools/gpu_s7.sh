#!/bin/bash
# Tonemapper: GPU tests (exact bytes, windowed == chain log-sum), diagnostics per log-sum mode,
# then the configuration bench lines and the multi-rank rehearsal (gpu_s6.sh's tail).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-s7}
mkdir -p $out
st=$out/status.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_tonemap.py -v -s -m gpu -x --timeout 200 --timeout-method thread > $out/pytest_tm.log 2>&1
rc=$?; echo "pytest tonemap rc=$rc" > $st
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 2 1 0; do
  RTG_TM_SEQSUM=$m timeout -k 10 300 python -u tools/diag_tonemap.py > $out/diag_tonemap_m$m.log 2>&1
  rc=$?; echo "diag_tonemap m$m rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for c in c2 c3 c3ton c4 c5; do
  timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
done
bash tools/gpu_multirank.sh ${1:-s7}
rc=$?; echo "multirank rc=$rc" >> $st
exit $rc
