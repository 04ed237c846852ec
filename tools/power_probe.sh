#!/usr/bin/env bash
# Diagnostic: package power / shader clock sampled every ~0.5 s (wall-clock
# stamped) while tools/power_probe.py runs each kernel variant back to back.
set -u
mkdir -p gpurun_out
( for i in $(seq 1 60); do
    echo "T $(date +%s.%N)"
    timeout 10 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk clock level"
    sleep 0.3
  done ) > gpurun_out/smi.log 2>&1 &
spid=$!
timeout -k 10 300 python tools/power_probe.py --external-smi --launches ${LAUNCHES:-60000} --variants ${PV:-0,3,4} > gpurun_out/pp.log 2>&1
rc=$?
kill $spid 2>/dev/null
wait $spid 2>/dev/null
echo "probe rc=$rc"
exit $rc
