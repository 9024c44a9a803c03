# Headline bench (parts prediction included) at 16 / 24 / 31 frames in flight, one hardware queue
# per replica stream + 1 (RTG_BENCH_HW_QUEUES; the box refuses more than 32)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05aa
for F in 16 24 31; do
  RTG_BENCH_HW_QUEUES=$((F + 1)) timeout -k 10 300 python bench.py --inflight $F --no-sweep --no-cpu-baseline > gpurun_out/r05aa/inflight_$F.log 2>&1 || exit $?
done
