#!/bin/bash
# Rehearsal of the driver's multi-GPU bench flow on a one-GPU box: torchrun with N ranks
# sharing GPU 0 (RTG_BENCH_BACKEND=gloo), image partition + shared-frame gather.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-mr}
mkdir -p $out
for n in 2 4; do
  RTG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) bench.py --gpus $n --steps 10 --warmup 2 > $out/bench_n$n.log 2>&1
  rc=$?; echo "n=$n rc=$rc" >> $out/status.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
