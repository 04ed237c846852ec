set -u
mkdir -p gpurun_out
for wk in "10 50" "1000 50" "10 2000" "3000 3000"; do
  set -- $wk
  timeout -k 10 300 python bench.py --warmup $1 --steps $2 --no-cpu --no-host > gpurun_out/warm_$1_$2.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/warm_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', d['roofline']['kernel_avg_us'], d['value'])"
done
