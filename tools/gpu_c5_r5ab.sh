#!/bin/bash
# C5 on the round-5 library (ab_r5/, git archive of the round-5 tree, built in place) against the
# current one on the same box, interleaved; current with and without the quantised child boxes.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-c5r5ab}
mkdir -p $out
args="--config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-sweep"
for rep in 1 2; do
  for v in r5 cur cur_noq; do
    echo "$(date +%T) start $v.$rep" >> $out/status.txt
    case $v in
      r5) (cd ab_r5 && timeout -k 10 300 python bench.py $args) > $out/$v.$rep.log 2>&1 ;;
      cur) timeout -k 10 300 python bench.py $args > $out/$v.$rep.log 2>&1 ;;
      cur_noq) RTG_QNODES=0 timeout -k 10 300 python bench.py $args > $out/$v.$rep.log 2>&1 ;;
    esac
    rc=$?; echo "$(date +%T) $v.$rep rc=$rc" >> $out/status.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
