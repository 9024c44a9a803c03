#!/bin/bash
# GPU-box check sequence: gpu tests, smoke, bench (sweep, CPU baseline), rocprofv3 kernel
# trace of the bench, then per K in {100352, 1002528} three separate PMC passes
# (FETCH_SIZE / WRITE_SIZE / TCC hit-miss-req), each its own rocprofv3 run.
# Usage (from this container): gpurun --timeout 1500 -- bash tools/gpu_check.sh <tag> [skip-tests]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" > $st
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --no-extras > $out/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
for K in 100352 1002528; do
  args="--steps 3 --warmup 1 --no-cpu-baseline --no-sweep --no-extras --K $K"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_fetch_$K -o run -- python bench.py $args > $out/pmc_fetch_$K.log 2>&1
  rc=$?; echo "pmc fetch $K rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_write_$K -o run -- python bench.py $args > $out/pmc_write_$K.log 2>&1
  rc=$?; echo "pmc write $K rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_tcc_$K -o run -- python bench.py $args > $out/pmc_tcc_$K.log 2>&1
  rc=$?; echo "pmc tcc $K rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $st
