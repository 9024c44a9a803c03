#!/bin/bash
# Round-3 GPU sequence: gpu tests + smoke, headline bench, kernel trace, and the limiter
# counters of the headline kernels -- one rocprofv3 --pmc pass per counter group (SQ issue /
# stall, SQ instruction mix + LDS, TCP (vL1D), TCC (L2)), each its own run.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r03.sh <tag> [skip-tests] [extra bench args]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r03}
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
shift
skip=0
if [ "$1" == "skip-tests" ]; then skip=1; shift; fi
extra="$@"
if [ $skip -eq 0 ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" > $st
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py $extra > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
# kernel trace of serial frames (--inflight 1): its per-kernel averages are the live event
# timings' (with frames in flight, overlapping kernels stretch each other's durations)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-sweep --no-extras $extra > $out/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $st
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1
args="--steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-sweep --no-extras $extra"
k=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
            "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
            "WRITE_SIZE" \
            "FETCH_SIZE" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-include-regex "rtg::k_" -f csv -d $out/pmc$k -o run -- python bench.py $args > $out/pmc$k.log 2>&1
  rc=$?; echo "pmc$k ($pass) rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $st
