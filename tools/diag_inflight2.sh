# Headline bench at (frames in flight, hardware queues) around the default (16, 17)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05ab
for FQ in 16:17 15:16 16:16 14:15 12:13; do
  F=${FQ%:*}; Q=${FQ#*:}
  RTG_BENCH_HW_QUEUES=$Q timeout -k 10 300 python bench.py --inflight $F --no-sweep --no-cpu-baseline > gpurun_out/r05ab/inflight_${F}_$Q.log 2>&1 || exit $?
done
