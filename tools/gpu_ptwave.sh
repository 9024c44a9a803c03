#!/bin/bash
# Wavefront path tracer: parity (pytest), fused vs wavefront timings (step kernel at 2 and 1
# waves per SIMD), C2 fused-kernel check after the node-step refactor.
set -o pipefail
OUT=gpurun_out/${1:-ptw}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pathtrace.py -k "wavefront or equals_oracle" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 240 python -u tools/diag_ptwave.py 1024 16 > $OUT/ptwave.log 2>&1 || { cat $OUT/ptwave.log; exit 1; }
cat $OUT/ptwave.log
RTGPU_LIB=$PWD/advanced-cpu-raytracing_amd/libpw1.so timeout -k 10 240 python -u tools/diag_ptwave.py 1024 16 > $OUT/ptwave_w1.log 2>&1 || { cat $OUT/ptwave_w1.log; exit 1; }
cat $OUT/ptwave_w1.log
timeout -k 10 120 python -u tools/diag_tree.py c2 > $OUT/c2.log 2>&1 || { cat $OUT/c2.log; exit 1; }
cat $OUT/c2.log
