cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; o=gpurun_out/r04n; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v -x --timeout 300 --timeout-method thread -s > $o/pytest_cfg.log 2>&1 &&
for c in c3 c3ton c4; do for e in base RTG_DEFER_ANY=0; do
  timeout -k 10 200 env ${e/base/X=1} python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-sweep --no-extras > $o/b_${c}_${e/=/_}.log 2>&1 || exit 1
done; done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c3 -o run -- python bench.py --config c3 --steps 5 --warmup 2 --inflight 1 --no-cpu-baseline --no-sweep --no-extras > $o/prof_c3.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/bench.log 2>&1
