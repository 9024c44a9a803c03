#!/bin/bash
# Configuration A/B over environment settings, interleaved twice, then the deferral tests.
# Usage: gpurun -- bash tools/gpu_env_ab.sh <tag>   with CONFIGS="c3 c4 ..." and
# ENV_AB="base NAME=VALUE[,NAME=VALUE] ..." in the environment (AB_TESTS: pytest selection).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
st=$out/status.txt
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -v -x --timeout 300 --timeout-method thread -s > $out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $st
  [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for setting in $ENV_AB; do
    name=${setting//[=,]/_}
    envs=(X_AB=1)
    [ "$setting" != base ] && IFS=, read -ra envs <<< "$setting"
    for c in ${CONFIGS:-headline}; do
      steps=40; [ $c != headline ] && steps=10
      timeout -k 10 200 env "${envs[@]}" python bench.py --config $c --steps $steps --warmup 3 --no-cpu-baseline --no-sweep --no-extras > $out/bench_${name}_${c}_$rep.log 2>&1
      rc=$?; echo "bench $name $c $rep rc=$rc" >> $st
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
