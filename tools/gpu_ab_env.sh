#!/bin/bash
# A/B of run-time settings (environment) on one build: for each "NAME=VALUE" argument (or
# "base" for none) the headline, C3, C3ton and C4 bench lines; then the GPU parity tests with
# the last setting.  Usage: gpurun -- bash tools/gpu_ab_env.sh <tag> base RTG_TILE_MAP=3 ...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
: > $st
last=""
for setting in "$@"; do
  name=${setting//=/_}
  if [ "$setting" = base ]; then envs=(); else envs=("$setting"); fi
  for c in headline c3 c3ton c4; do
    steps=20; [ $c != headline ] && steps=5
    env "${envs[@]}" timeout -k 10 300 python bench.py --config $c --steps $steps --warmup 2 --no-cpu-baseline --no-sweep --no-extras > $out/bench_${name}_$c.log 2>&1
    rc=$?; echo "bench $setting $c rc=$rc" >> $st
    [ $rc -ne 0 ] && exit $rc
  done
  last=$setting
done
if [ "$last" != base ] && [ -n "$last" ]; then envs=("$last"); else envs=(); fi
env "${envs[@]}" timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $out/pytest_last.log 2>&1
rc=$?; echo "pytest ($last) rc=$rc" >> $st
exit $rc
