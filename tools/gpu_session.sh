#!/usr/bin/env bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/timeout/signal stops the
# session (no further GPU work), a plain test failure (rc 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS="${STEPS:-smoke tests bench prof}"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session.log
  tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  if [ $rc -ne 0 ] && [ -n "${STOP_ON_FAIL:-}" ]; then echo "stopping after a failure (STOP_ON_FAIL)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests ${T_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${T_ARGS:-} ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    bench5) run bench5 600 python bench.py --config c5 --no-cpu ;;
    bench3) run bench3 600 python bench.py --config c3 --no-cpu --no-host ;;
    bench4) run bench4 600 python bench.py --config c4 --no-cpu --no-host ;;
    cfgs) for c in ${CFGS:-c3 c2b1536 c4 c5}; do run bench_$c 600 python bench.py --config $c --no-cpu --no-host ${CFG_ARGS:-}; done ;;
    pmc) run pmc 1100 bash tools/pmc_session.sh ;;
    stamps) for v in ${SV:-5 6}; do run stamps_${SCFG:-c2}_v$v 300 python tools/stamps.py ${SCFG:-c2} $v ${SW:-12}; done ;;
    tprobe) run tprobe 300 python tools/timing_probe.py ;;
    sweep) run sweep 300 python tools/probe_sweep.py ;;
    kbench) run kbench_${KCFG:-c2} ${KB_TIMEOUT:-600} python tools/kbench.py --config ${KCFG:-c2} --variants ${KV:-0,1,2,3,4,5} ${KB_ARGS:-} ;;
    kbench5) run kbench5 600 python tools/kbench.py --config c5 --variants ${KV:-0,1} ;;
    bench3h) run bench3h 600 python bench.py --config c3 --host-sweep --cpu-seconds 2 ;;
    sweepab) run sweep_zc0 600 env HDFS_CRC32C_ZERO_COPY_KB=0 python bench.py --config c3 --host-sweep --no-cpu --steps 200 --warmup 50 && run sweep_zc 600 python bench.py --config c3 --host-sweep --no-cpu --steps 200 --warmup 50 ;;
    brate) run brate 300 tools/block_rate ${BR_ARGS:-16 400 16 30} ;;
    brateab) run brate_rec 300 env HDFS_CRC32C_QUEUE_RECORD=1 tools/block_rate ${BR_ARGS:-16 400 16 30} && run brate 300 tools/block_rate ${BR_ARGS:-16 400 16 30} ;;
    ab02) for c in ${ABCFGS:-c5 c2b1536}; do
            run ab_r02_$c 600 bash -c "cd scratch/r02 && python bench.py --config $c --no-cpu --no-host" &&
            run ab_head_$c 600 python bench.py --config $c --no-cpu --no-host; done ;;
    bsweep) for spin in ${BSPIN:-50 0}; do for mb in ${BMB:-8 16 32}; do for th in ${BTH:-16 32}; do
              run bsw_s${spin}_mb${mb}_t${th} 120 env HDFS_CRC32C_QUEUE_SPIN_US=$spin tools/block_rate $th 300 $mb ${BWIN:-30} 4 1;
            done; done; done ;;
    btrace) for th in ${BTH:-4 16}; do run btrace_t$th 120 env HDFS_CRC32C_QUEUE_TRACE=gpurun_out/qtrace_t$th.jsonl tools/block_rate $th 300 16 30 4 1; done ;;
    bpoll) for v in ${BPV:-p1 p5 p20 sync rec}; do
             case $v in tim) E="HDFS_CRC32C_QUEUE_TIMING=1";; rec) E="HDFS_CRC32C_QUEUE_RECORD=1";; rectim) E="HDFS_CRC32C_QUEUE_RECORD=1 HDFS_CRC32C_QUEUE_TIMING=1";; s*) E="HDFS_CRC32C_QUEUE_SPIN_US=${v#s}";; p*) E="HDFS_CRC32C_QUEUE_POLL_US=${v#p}";; esac
             run bpoll_$v 120 env $E HDFS_CRC32C_QUEUE_TRACE=gpurun_out/qtrace_$v.jsonl tools/block_rate ${BPT:-16} 300 16 30 4 1; done ;;
    abwt) for c in ${ABCFGS:-c2b1000 c2b1536}; do
            run abwt_base_$c 600 bash -c "cd scratch/wt && python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-}" &&
            run abwt_head_$c 600 python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-}; done ;;
    abwt2) for c in ${ABCFGS:-c2b1000 c2b1536}; do
            run abwt2_base_$c 600 python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-} &&
            run abwt2_cand_$c 600 bash -c "cd scratch/wt2 && python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-}"; done ;;
    abwt3) for c in ${ABCFGS:-c2b1000 c2b1536}; do
            run abwt3_base_$c 600 python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-} &&
            run abwt3_cand_$c 600 bash -c "cd scratch/wt3 && python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-}"; done ;;
    qsum) run qsum 60 bash -c 'for f in gpurun_out/qtrace_*.jsonl; do echo "$f"; python tools/qtrace_summary.py "$f"; done' ;;
    bq) run bq_t16_mb16 300 tools/block_rate 16 400 16 30 4 0 &&
        run bq_t16_mb32 200 tools/block_rate 16 300 32 30 4 1 &&
        run bq_t32_mb16 200 tools/block_rate 32 300 16 30 2 1 &&
        run bq_t32_mb32 200 tools/block_rate 32 300 32 30 2 1 ;;
    bqprof) run bq_mb8 200 tools/block_rate 16 400 8 30 1 1 &&
            run bq_prof 300 rocprofv3 --kernel-trace --stats -d $OUT/bq_prof -o run --output-format csv -- tools/block_rate 16 100 16 30 2 1 ;;
    bqs) for ns in 1 2; do
           run bqs${ns}_t16_mb16 200 env HDFS_CRC32C_QUEUE_STREAMS=$ns tools/block_rate 16 400 16 30 2 1 &&
           run bqs${ns}_t16_mb8 200 env HDFS_CRC32C_QUEUE_STREAMS=$ns tools/block_rate 16 400 8 30 2 1 &&
           run bqs${ns}_t32_mb16 200 env HDFS_CRC32C_QUEUE_STREAMS=$ns tools/block_rate 32 300 16 30 1 1 || break; done ;;
    gabl) run kbench_gabl_c2b1000 400 python tools/kbench.py --config c2b1000 --variants 0,3,4,70,71,72,73,74 &&
          run kbench_gabl_c2b1536 400 python tools/kbench.py --config c2b1536 --variants 0,3,4,70,72,73 &&
          run kbench_gabl_c2 300 python tools/kbench.py --config c2 --variants 0,3,4 ;;
    cgroup) run cgroup 30 bash -c 'cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat; nproc; cat /proc/self/status | grep -i cpus_allowed_list' ;;
    lsp) run lsp 120 tools/launch_stop_probe ;;
    c4model) run c4model 300 python tools/c4_model.py ;;
    stash) for b in ${SB:-basewt stashwt stashB}; do run stash_$b 300 python tools/stash_repro.py $b ${SBPC:-4,7,100,1000,1536}; done ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
            python3 bench.py --no-cpu --no-host ;;
  esac
done
echo "session done"
