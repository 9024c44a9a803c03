#!/bin/bash
# Development loop on the GPU box: chosen test files (default: all gpu tests), then one
# headline bench line (no sweep / CPU baseline) and optional extra bench args.
# Usage: gpu_dev.sh <tag> "<pytest targets>" ["<bench args>"]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-dev}
mkdir -p $out
targets=${2:-tests}
timeout -k 10 900 python -u -m pytest $targets -q -m gpu -x --timeout 300 --timeout-method thread -s > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $out/status.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --no-extras $3 > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $out/status.txt
exit $rc
