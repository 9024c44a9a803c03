#!/bin/bash
# Quick GPU iteration: parity tests, bench, kernel trace, one SQ counter pass.
# Usage: gpurun --timeout 900 -- bash tools/gpu_perf.sh <tag>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-perf}
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $st
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_sq -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc" >> $st
exit 0
