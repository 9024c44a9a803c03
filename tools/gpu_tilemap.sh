#!/bin/bash
# Tile-map experiment: bench under each RTG_TILE_MAP mode.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-tm}
mkdir -p $out
for m in 0 1 2; do
  RTG_TILE_MAP=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/bench_m$m.log 2>&1 || exit 1
done
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $out/pytest.log 2>&1
echo "pytest rc=$?" > $out/status.txt
