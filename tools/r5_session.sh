#!/usr/bin/env bash
# Round-5 GPU session steps (each step under its own time limit; a crash,
# timeout or signal ends the session).  STEPS selects them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STEPS:-calls multi}; do
  case $s in
    calls) run calls 120 tools/launch_rate calls 64 4000 ;;
    brate) run brate 240 tools/block_rate ${BR_ARGS:-16 400 16 30 2 1} ;;
    brate1) run brate1 120 tools/block_rate 1 2000 16 0 1 1 ;;
    bres) run bres12 240 tools/block_rate 16 400 16 30 2 1 && run bres16 240 env HDFS_CRC32C_RESIDENT_WAVES=16 tools/block_rate 16 400 16 30 2 1 &&
          run bres1_16 120 env HDFS_CRC32C_RESIDENT_WAVES=16 tools/block_rate 1 2000 16 0 1 1 ;;
    bresall) for w in 12 16 12x11 16x15; do run bres_$w 240 env HDFS_CRC32C_RESIDENT_WAVES=$w tools/block_rate 16 400 16 30 2 1 &&
               run bres1_$w 120 env HDFS_CRC32C_RESIDENT_WAVES=$w tools/block_rate 1 2000 16 0 1 1 || exit 1; done ;;
    bqblock) run bq_spin 240 tools/block_rate 16 400 16 30 2 1 && run bq_block 240 env HDFS_CRC32C_QUEUE_BLOCKING=1 tools/block_rate 16 400 16 30 2 1 &&
             run bq_spin32 240 tools/block_rate 32 200 32 30 1 1 && run bq_block32 240 env HDFS_CRC32C_QUEUE_BLOCKING=1 tools/block_rate 32 200 32 30 1 1 ;;
    btrace) run btrace1 120 env HDFS_CRC32C_RESIDENT_STAMPS=1 HDFS_CRC32C_RESIDENT_WAVES=16 tools/block_rate 1 2000 16 0 1 1 &&
            run btrace16 240 env HDFS_CRC32C_RESIDENT_STAMPS=1 HDFS_CRC32C_RESIDENT_WAVES=16 tools/block_rate 16 400 16 30 2 1 ;;
    rtt) run rtt 120 tools/launch_rate rtt 2000 ;;
    brlong) run brlong 300 tools/block_rate 16 4000 16 30 2 1 ;;
    bspin) for sp in 50 10 0; do run bspin$sp 200 env HDFS_CRC32C_QUEUE_SPIN_US=$sp tools/block_rate 16 400 16 30 2 1 || exit 1; done ;;
    b4) run bench_c4 300 python bench.py --config c4 --no-cpu --no-host --steps 200 --warmup 20 ;;
    tres) run tres 200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "resident or destroyed" ;;
    multi) run multi 180 tools/launch_rate multi 256 2000 ;;
    multiprof) run multiprof 300 rocprofv3 --kernel-trace --hip-trace --stats -d $OUT/multiprof -o run --output-format csv -- tools/launch_rate multi 256 1000 ;;
    tmulti) run tmulti 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "multi" ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    bench20) run bench20 600 python bench.py --steps 20 --warmup 5 ;;
    b20x3) for r in 1 2 3; do run bench20_$r 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-host || exit 1; done ;;
    c3x20) run c3_20 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu --no-host && run c3_2000 300 python bench.py --config c3 --no-cpu --no-host ;;
    c4model) run c4model 300 python tools/c4_model.py ;;
    tgen) run tgen 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "general or golden or random or fuzz or mixed or unaligned or shifted or verify or write_plan or fsx or edge or small" ;;
    tqueue) run tqueue 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "block_queue or overlapping or per_launch or destroyed or across_streams or recycled" ;;
    tgench) for n in 5 21 31; do run tgen_gch$n 600 env HDFS_CRC32C_GCHUNKS=$n python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "general or golden or random or fuzz or mixed or edge" || exit 1; done ;;
    g1000) run g1000_base 300 python bench.py --config c2b1000 --no-cpu --no-host &&
           run g1000_16 300 env HDFS_CRC32C_GCHUNKS_DIV=16 python bench.py --config c2b1000 --no-cpu --no-host &&
           run g1000_32 300 env HDFS_CRC32C_GCHUNKS_DIV=24 python bench.py --config c2b1000 --no-cpu --no-host &&
           run g1000_16io 300 env HDFS_CRC32C_GCHUNKS_DIV=16 HDFS_CRC32C_PADDED_FULL=0 python bench.py --config c2b1000 --no-cpu --no-host &&
           run g1000_24io 300 env HDFS_CRC32C_GCHUNKS_DIV=24 HDFS_CRC32C_PADDED_FULL=0 python bench.py --config c2b1000 --no-cpu --no-host &&
           run g1000_base2 300 python bench.py --config c2b1000 --no-cpu --no-host ;;
    tg1000) run tg1000 600 env HDFS_CRC32C_GCHUNKS_DIV=24 HDFS_CRC32C_PADDED_FULL=0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "general or golden or random or fuzz or mixed or edge" ;;
    gblk) for c in ${GBCFGS:-c2b1000 c2b700 c2b2560 c2b3000 c2b4000 c2b1536}; do for gb in ${GBS:-0 48}; do
             run gb_${c}_$gb 300 env HDFS_CRC32C_GBLOCKS=$gb python bench.py --config $c --no-cpu --no-host || exit 1; done; done ;;
    tgblk) run tgblk 600 env HDFS_CRC32C_GBLOCKS=48 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "general or golden or random or fuzz or mixed or edge" ;;
    gch) for n in ${GCH:-16 5 10 21 16}; do run gch_${n} 300 env HDFS_CRC32C_GCHUNKS=$n python bench.py --config ${GCFG:-c2b1536} --no-cpu --no-host || exit 1; done ;;
    soak) run soak $(( ${SOAK_S:-240} + 90 )) python -u tools/soak.py --seconds ${SOAK_S:-240} --out $OUT/soak.jsonl ;;
    syncp) run sync_default 120 python tools/sync_probe.py && run sync_spin 120 python tools/sync_probe.py --spin ;;
    tbenchq) run tbenchq 900 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread ;;
    tverify) run tverify 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "verify or bitmap or overlapping" ;;
    fcp) run fcp 600 python -u tools/fixed_cost_probe.py --rounds ${FCP_ROUNDS:-3} ;;
    tres5) run tres5 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "resident or block_queue" ;;
    brate5) run brate5 400 tools/block_rate 16 400 16 30 2 1 ;;
    tall) run tall 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    callsab) for r in 1 2 3; do run calls_base_$r 120 abwt/tools/launch_rate calls 64 4000 && run calls_cand_$r 120 tools/launch_rate calls 64 4000 || exit 1; done ;;
    kb16) run kb16_p2048 300 python tools/kbench.py --config p2048 --variants 0,2 --rounds 9 --iters 300 &&
          run kb16_c2 300 python tools/kbench.py --config c2 --variants 0,2 --rounds 7 --iters 300 ;;
    halvestrace) run halvestrace 300 rocprofv3 --kernel-trace -d $OUT/halvestrace -o run --output-format csv -- python3 tools/fixed_cost_probe.py --modes c2,c2_halves --rounds 1 --steps 300 ;;
    calls4) for r in 1 2; do for w in abwt abwt_noatomic abwt_wg .; do n=$(basename $w); run calls_${n}_$r 120 $w/tools/launch_rate calls 64 4000 || exit 1; done; done ;;
    tstream) run tstream 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "destroyed or recycled or context" ;;
    pmcg) for c in ${PMCCFGS:-c2 c2b1000 c2b700}; do run pmc_$c 900 env PMC_CONFIG=$c PMC_OUT=$OUT/pmc_$c bash tools/pmc_session.sh || exit 1; done ;;
    tmulti5) run tmulti5 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "multi" ;;
    calls2) for r in 1 2; do run calls_base_$r 120 abwt/tools/launch_rate calls 64 4000 && run calls_head_$r 120 tools/launch_rate calls 64 4000 || exit 1; done ;;
    prof5) run prof5 600 rocprofv3 --kernel-trace --stats -d $OUT/prof5 -o run --output-format csv -- python3 bench.py --no-config4 --no-strong ;;
    prof5d) run prof5d 600 rocprofv3 --kernel-trace --stats -d $OUT/prof5d -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 ;;
    kbhoist) for c in ${KBCFGS:-c2b1000 c2b700 c2b1536}; do run kbh_$c 300 python tools/kbench.py --config $c --variants ${KBV:-0,49,75,2} --rounds 9 --iters 300 || exit 1; done ;;
    benchd) run benchd 600 python bench.py --steps 20 --warmup 5 ;;
    tpad) run tpad 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "padded or general or golden or random or fuzz or mixed or edge or small or verify or write_plan" ;;
    padw) for c in ${PADWCFGS:-c2w1000 c2w2000 c2w4000 c2w700 c2w100 c2b2048}; do
             run padw_gen_$c 300 env HDFS_CRC32C_PADDED_TILES=0 python bench.py --config $c --no-cpu --no-host &&
             run padw_tile_$c 300 python bench.py --config $c --no-cpu --no-host || exit 1; done ;;
    kbgen) for c in ${KBGCFGS:-c2 c2b2048 c2w2000}; do run kbg_$c 300 python tools/kbench.py --config $c --variants ${KBGV:-0,49,79,62} --rounds 7 --iters 300 || exit 1; done ;;
    kbovl) for c in ${KBOCFGS:-c2 p2048 c5 p1024}; do run kbo_$c 300 python tools/kbench.py --config $c --variants ${KBOV:-0,62,80} --rounds 9 --iters 300 || exit 1; done ;;
    halfab) for c in ${HALFCFGS:-c2b700 c2b600 c2b768 c2b100 c2b200 c2w700 c2b1100 c2b1280}; do
             run halfab_off_$c 300 env HDFS_CRC32C_HALF_TILES=0 python bench.py --config $c --no-cpu --no-host &&
             run halfab_on_$c 300 python bench.py --config $c --no-cpu --no-host || exit 1; done ;;
    thalf) run thalf 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "half or padded or general or golden or random or fuzz or mixed or edge or small or verify or write_plan" ;;
    abhalf) for r in $(seq 1 ${ABR:-2}); do for c in ${ABHCFGS:-c2b1000 c2b2000 c2t c2u c2b1536 c2}; do
             run abh_base_${c}_$r 300 python abwt/bench.py --config $c --no-cpu --no-host &&
             run abh_cand_${c}_$r 300 python bench.py --config $c --no-cpu --no-host || exit 1; done; done ;;
    tailab) for r in 1 2; do for c in ${TAILCFGS:-c2b1000 c2b2000 c2b4000}; do
             run tailab_item_${c}_$r 300 python bench.py --config $c --no-cpu --no-host &&
             run tailab_gen_${c}_$r 300 env HDFS_CRC32C_PADDED_TAIL_GEN=1 python bench.py --config $c --no-cpu --no-host || exit 1; done; done ;;
    p2tail) for r in 1 2; do for c in ${P2CFGS:-c2t c5}; do
             run p2t_item_${c}_$r 300 python bench.py --config $c --no-cpu --no-host &&
             run p2t_gen_${c}_$r 300 env HDFS_CRC32C_POW2_TAIL_GEN=1 python bench.py --config $c --no-cpu --no-host || exit 1; done; done ;;
    htail) for c in ${HTCFGS:-c2b700 c2b1100 c2b100 c2b600}; do
             run ht_rule_$c 300 python bench.py --config $c --no-cpu --no-host &&
             run ht_never_$c 300 env HDFS_CRC32C_HALF_TAIL_GEN=0 python bench.py --config $c --no-cpu --no-host &&
             run ht_always_$c 300 env HDFS_CRC32C_HALF_TAIL_GEN=1 python bench.py --config $c --no-cpu --no-host || exit 1; done ;;
    padab) for r in $(seq 1 ${PADR:-1}); do for c in ${PADCFGS:-c2b1000 c2b700 c2b4000 c2b2000 c2b100}; do
             run padab_gen_${c}_$r 300 env HDFS_CRC32C_PADDED_TILES=0 python bench.py --config $c --no-cpu --no-host &&
             run padab_tile_${c}_$r 300 python bench.py --config $c --no-cpu --no-host || exit 1; done; done ;;
    c4x20) for r in 1 2; do run c4_20_$r 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu --no-host || exit 1; done ;;
    tbench) run tbench 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread ;;
    configs) for c in ${CFGS:-c3 c4 c5 c2b1536 c2b1000 c2t c2u c3u}; do run cfg_$c 300 python bench.py --config $c --no-cpu --no-host || exit 1; done ;;
    prof2) run prof2 600 rocprofv3 --kernel-trace --stats -d $OUT/prof2 -o run --output-format csv -- python3 bench.py ;;
    prof3) run prof3 300 rocprofv3 --kernel-trace --stats -d $OUT/prof3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu --no-host ;;
    pmc3) run pmc3 900 env PMC_CONFIG=c3 PMC_OUT=$OUT/pmc_c3 bash tools/pmc_session.sh ;;
    pmc2) run pmc2 900 env PMC_CONFIG=c2 PMC_OUT=$OUT/pmc_c2 bash tools/pmc_session.sh ;;
    ab) for r in $(seq 1 ${ABROUNDS:-1}); do for c in ${ABCFGS:-c2b1000 c2b1536 c2t c2u c5}; do
          run ab_cand_${c}_$r 300 python bench.py --config $c --no-cpu --no-host ${AB_ARGS:-} || exit 1; done; done ;;
  esac
done
echo "session done"
