#!/bin/bash
# SQ issue/stall counters for the headline kernels (one pass), plus the counter list.
# Usage: gpurun -- bash tools/gpu_sq.sh <tag> [bench args]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "rtg::k_" -f csv -d $out/pmc_sq -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $out/pmc_sq.log 2>&1
rc=$?; echo "sq rc=$rc" > $out/status.txt
exit $rc
