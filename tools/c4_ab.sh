#!/usr/bin/env bash
# Config 4 A/B on one GPU: pipelined multi-plan steps (CRC32C_MULTI_PIPELINE,
# the default) against every step in stream order (BENCH_C4_PIPELINE=0),
# interleaved, in the driver's 20-step window and over 2000 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/c4ab}
mkdir -p "$OUT"
for rep in ${REPS:-1 2}; do
  for pipe in 1 0; do
    for steps in ${STEPS_LIST:-20 2000}; do
      w=$([ "$steps" -gt 100 ] && echo 500 || echo 5)
      f=$OUT/c4_p${pipe}_s${steps}_r${rep}.json
      BENCH_C4_PIPELINE=$pipe timeout -k 10 300 python bench.py --config c4 --steps "$steps" --warmup "$w" \
        --no-cpu --no-host > "$f" 2> "$f.err"
      rc=$?
      echo "pipe=$pipe steps=$steps rep=$rep rc=$rc"
      [ $rc -ne 0 ] && { tail -5 "$f.err"; exit $rc; }
      python - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
c = json.loads(l)["config4"]
print("  kernel_step_us %.3f  500: %s  shard %.3f  exact %s  %s" % (c["kernel_step_us"], c["kernel_step_us_500"],
      c["shard_kernel_us"], c["bit_exact"], c["launch"]))
PY
    done
  done
done
