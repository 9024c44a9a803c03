#!/bin/bash
# GPU-box check sequence: gpu tests, smoke, bench (+sweep, CPU baseline), rocprofv3 kernel
# trace of the bench, PMC FETCH_SIZE / WRITE_SIZE passes.
# Usage (from this container): gpurun --timeout 1500 -- bash tools/gpu_check.sh <tag>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
timeout -k 10 900 python -m pytest tests -q -m gpu > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $st
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --sweep > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_write -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $out/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc" >> $st
