#!/bin/bash
# GPU-box check sequence: gpu tests, smoke, bench, rocprofv3 kernel trace, PMC passes.
# Usage (from this container): gpurun --timeout 1200 -- bash tools/gpu_check.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
st=gpurun_out/status3.txt
timeout -k 10 900 python -m pytest tests -q -m gpu -s > gpurun_out/pytest_gpu3.log 2>&1
rc=$?; echo "pytest rc=$rc" > $st
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke3.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --sweep > gpurun_out/bench3.log 2>&1
rc=$?; echo "bench rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof3.log 2>&1
rc=$?; echo "prof rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rtg::k_" -f csv -d gpurun_out/pmc3_fetch -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc3_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "rtg::k_" -f csv -d gpurun_out/pmc3_write -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc3_write.log 2>&1
rc=$?; echo "pmc write rc=$rc" >> $st
