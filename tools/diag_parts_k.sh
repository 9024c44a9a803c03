cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05t
for K in 1000 10000 100352; do
  timeout -k 10 300 python bench.py --K $K --steps 40 --no-sweep --no-cpu-baseline > gpurun_out/r05t/parts_K$K.log 2>&1 || exit $?
done
