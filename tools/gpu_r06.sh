#!/bin/bash
# Round-6 GPU sequence.  Usage: gpurun --timeout 1200 -- bash tools/gpu_r06.sh <tag> <step>... [-- bench args]
# steps: tests (pytest -m gpu + smoke), slivers (tools/diag_slivers.py), bench, prof (kernel
# trace of serial frames), pmc (limiter + HBM counter passes, one rocprofv3 --pmc run each),
# configs (bench --config c2..c5), ab (tools/gpu_ab_head.sh over the libraries in $AB_LIBS,
# e.g. AB_LIBS="base libpk2.so"), py:<name> (tools/<name>.py), envbench / envpy:<name> (bench.py /
# tools/<name>.py once per setting of $ENV_AB).  Every step has its own
# time limit; the first failing step ends the script.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
st=$out/status.txt
: > $st
steps=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do steps+=("$1"); shift; done
[ "$1" == "--" ] && shift
extra="$@"
run() {   # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "$(date +%T) start $name" >> $st
  timeout -k 10 $to "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $st
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in "${steps[@]}"; do
  case $s in
    tests)
      run pytest 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -s
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    tests:*)
      # one test file (tests/<name>.py)
      t=${s#tests:}
      run pytest_$t 600 python -u -m pytest tests/$t.py -v -m gpu -x --timeout 300 --timeout-method thread ;;
    slivers)
      run slivers 600 python -u tools/diag_slivers.py $out/slivers.json ;;
    bench)
      run bench 600 python bench.py $extra ;;
    prof)
      run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-sweep --no-extras $extra ;;
    trace:*)
      # kernel trace of a configuration's bench run with its frame parts, grouped by grid size
      c=${s#trace:}
      run trace_$c 600 rocprofv3 --kernel-trace --output-format csv -d $out/trace_$c -o run -- python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline $extra
      run groups_$c 120 python tools/trace_groups.py $out/trace_$c/run_kernel_trace.csv $out/trace_$c/groups.txt
      find $out/trace_$c -name "*kernel_trace.csv" -delete ;;
    ptrace:*)
      # a configuration's frame and its parts of 8 rendered one at a time (tools/diag_parts_serial.py),
      # kernel-traced and grouped by grid size
      c=${s#ptrace:}
      run ptrace_$c 400 rocprofv3 --kernel-trace --output-format csv -d $PWD/$out/ptrace_$c -o run -- python tools/diag_parts_serial.py $c 8 10
      run pgroups_$c 120 python tools/trace_groups.py $out/ptrace_$c/run_kernel_trace.csv $out/ptrace_$c/groups.txt
      find $out/ptrace_$c -name "*kernel_trace.csv" -delete ;;
    pmc|pmc:*)
      # counter passes (one rocprofv3 --pmc run per group) + one kernel-trace pass of the same
      # bench invocation; pmc:<name> puts them under $out/pmc_<name>/ (tools/pmc_kernels.py)
      name=${s#pmc}; name=${name#:}
      pd=$out/pmc${name:+_$name}
      mkdir -p $pd
      # pmc:c3 -> --config c3; pmc:K1002528 -> --K 1002528; pmc / pmc:headline -> the headline
      cfgarg=""
      case $name in c2|c3|c3ton|c4|c5) cfgarg="--config $name" ;; K*) cfgarg="--K ${name#K}" ;; esac
      args="--steps ${PMC_STEPS:-3} --warmup 1 --inflight 1 --no-cpu-baseline --no-sweep --no-extras $cfgarg $extra"
      k=0
      for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
                  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
                  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
                  "WRITE_SIZE" \
                  "FETCH_SIZE" \
                  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
        k=$((k+1))
        echo "$(date +%T) start pmc$name/$k" >> $st
        timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $pass --kernel-include-regex "rtg::k_" -f csv -d $pd/pmc$k -o run -- python bench.py $args > $pd/pmc$k.log 2>&1
        rc=$?; echo "$(date +%T) pmc$name/$k ($pass) rc=$rc" >> $st
        if [ $rc -ne 0 ]; then exit $rc; fi
      done
      echo "$(date +%T) start kt$name" >> $st
      timeout -k 10 ${PMC_TIMEOUT:-120} rocprofv3 --kernel-trace --stats -f csv -d $pd/kt -o run -- python bench.py $args > $pd/kt.log 2>&1
      rc=$?; echo "$(date +%T) kt$name rc=$rc" >> $st
      if [ $rc -ne 0 ]; then exit $rc; fi
      # summarise on the box and drop the per-dispatch CSVs (gpurun copies back at most 64 MiB)
      wl=headline; K=100352
      case $name in c2|c3|c3ton|c4|c5) wl=$name; K=0 ;; K*) K=${name#K} ;; esac
      python tools/pmc_kernels.py $pd $pd/summary.json --workload $wl --K $K > $pd/summary.log 2>&1
      rc=$?; echo "$(date +%T) summary$name rc=$rc" >> $st
      find $pd -name "*counter_collection.csv" -delete
      find $pd -name "*kernel_trace.csv" -delete
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    configs)
      # $CFGS: the configurations (default all); $CFG_CPU=1 keeps each line's cpu_baseline
      cpu="--no-cpu-baseline"; [ -n "$CFG_CPU" ] && cpu=""
      for c in ${CFGS:-c2 c3 c3ton c4 c5}; do
        if [ $c == c5 ]; then
          run cfg_c5 600 python bench.py --config c5 --steps 5 --warmup 1 $cpu $extra
        else
          run cfg_$c 400 python bench.py --config $c $cpu $extra
        fi
      done ;;
    inflight:*)
      # one configuration at several frames in flight ($INFLIGHT, default 1 2 4)
      c=${s#inflight:}
      for f in ${INFLIGHT:-1 2 4}; do
        run inflight_${c}_$f 600 python bench.py --config $c --inflight $f --steps ${CFG_STEPS:-4} --warmup 1 --no-extras --no-cpu-baseline --no-sweep $extra
      done ;;
    abparts)
      # library A/B ($AB_LIBS, "base" = librtgpu.so) on one configuration ($ABCFG, default c3) with
      # its parts (bench extras), twice interleaved, then each library's serial parts (diag_parts_serial)
      for rep in 1 2; do
        for l in $AB_LIBS; do
          lib=""; [ $l != base ] && lib=$PWD/advanced-cpu-raytracing_amd/$l
          run abparts_${l}_$rep 400 env RTGPU_LIB=$lib python bench.py --config ${ABCFG:-c3} --no-cpu-baseline --no-sweep --steps 10 $extra
        done
      done
      for l in $AB_LIBS; do
        lib=""; [ $l != base ] && lib=$PWD/advanced-cpu-raytracing_amd/$l
        run abserial_$l 300 env RTGPU_LIB=$lib python tools/diag_parts_serial.py ${ABCFG:-c3} 8 10
      done ;;
    ab)
      run ab 1500 bash tools/gpu_ab_head.sh $tag/ab $AB_LIBS ;;
    multirank)
      # the driver's N-rank launch rehearsed on one GPU (gloo; ranks share GPU 0)
      run multirank_n2 400 env RTG_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 2 ;;
    envbench)
      # the headline bench (with gather / host-frame / parts / ordered extras) once per setting in
      # $ENV_AB ("base" or NAME=VALUE[,NAME=VALUE])
      for setting in $ENV_AB; do
        name=$(echo "$setting" | tr "=,/" "___")
        envs=()
        [ "$setting" != base ] && IFS=, read -ra envs <<< "$setting"
        run envbench_$name 300 env "${envs[@]}" python bench.py --no-sweep --no-cpu-baseline $extra
      done ;;
    envcfg:*)
      # bench.py --config <c> (no extras) once per setting in $ENV_AB, twice interleaved
      c=${s#envcfg:}
      for rep in 1 2; do
        for setting in $ENV_AB; do
          name=$(echo "$setting" | tr "=,/" "___")
          envs=()
          [ "$setting" != base ] && IFS=, read -ra envs <<< "$setting"
          run envcfg_${c}_${name}_$rep 400 env "${envs[@]}" python bench.py --config $c --no-extras --no-cpu-baseline --steps ${CFG_STEPS:-10} $extra
        done
      done ;;
    envpy:*)
      # tools/<name>.py once per setting in $ENV_AB
      t=${s#envpy:}
      for setting in $ENV_AB; do
        name=$(echo "$setting" | tr "=,/" "___")
        envs=()
        [ "$setting" != base ] && IFS=, read -ra envs <<< "$setting"
        run ${t}_$name 300 env "${envs[@]}" python -u tools/$t.py
      done ;;
    py:*)
      t=${s#py:}
      run $t 600 python -u tools/$t.py ;;
    *)
      echo "unknown step $s" >> $st; exit 2 ;;
  esac
done
echo done >> $st
