#!/bin/bash
# Any-hit tree A/B: shadow tests, then the headline and C3 / C3-ton / C4 benches per RTG_AHB mode
# (split = default, exact, ref), and the part diagnostics.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-ahb}
mkdir -p $out
st=$out/status.txt
RTG_AHB_VERBOSE=1 timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $st
if [ $rc -ne 0 ]; then exit $rc; fi
for mode in exact split ref; do
  RTG_AHB=$mode RTG_AHB_VERBOSE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --no-extras > $out/bench_$mode.log 2>&1
  rc=$?; echo "bench $mode rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
  for c in c3 c3ton c4; do
    RTG_AHB=$mode RTG_AHB_VERBOSE=1 timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $out/bench_${c}_$mode.log 2>&1
    rc=$?; echo "bench $c $mode rc=$rc" >> $st
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
timeout -k 10 240 python -u tools/diag_parts.py 20 > $out/diag_parts.log 2>&1
rc=$?; echo "diag_parts rc=$rc" >> $st
echo done >> $st
