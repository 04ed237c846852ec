set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/stamps.py c2 25 > gpurun_out/stamps_v25.log 2>&1 || exit $?
HDFS_CRC32C_TAIL_STEAL=1 HDFS_CRC32C_KVARIANT=26 timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/tests26.log 2>&1; rc=$?; echo "tests26 steal rc=$rc"; tail -3 gpurun_out/tests26.log
if [ $rc -ne 0 ]; then exit $rc; fi
for st in 0 1; do for tl in 4 8 16; do
  HDFS_CRC32C_TAIL_STEAL=$st HDFS_CRC32C_TAIL=$tl timeout -k 10 300 python tools/kbench.py --config c2 --variants 17,26 --rounds 5 > gpurun_out/kbench_s${st}_t$tl.log 2>&1 || exit $?
done; done
HDFS_CRC32C_TAIL=8 timeout -k 10 300 python tools/stamps.py c2 28 > gpurun_out/stamps_v28.log 2>&1 || exit $?
echo done
