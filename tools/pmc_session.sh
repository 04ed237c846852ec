#!/usr/bin/env bash
# PMC counter passes for the CRC32C kernel (one rocprofv3 run per pass,
# kernel-trace only beside --pmc).  Workload: tools/kbench.py, one variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="${PMC_OUT:-gpurun_out/pmc}"
mkdir -p $OUT
export TMPDIR=/tmp
V="${PMC_VARIANT:-0}"
CFG="${PMC_CONFIG:-c2}"
WL="python3 tools/kbench.py --variants $V --rounds 1 --iters 10 --config $CFG"
pass() {  # name counters...
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o p --output-format csv -- $WL > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  tail -3 $OUT/$name.log
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
echo "pmc done"
