set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 21 24; do
  HDFS_CRC32C_KVARIANT=$v timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "golden or variant or crc32" > gpurun_out/t$v.log 2>&1; rc=$?; echo "tests $v rc=$rc"; tail -1 gpurun_out/t$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 300 python tools/kbench.py --config c2 --variants 0,21,24,2,4,22,19 > gpurun_out/kbench.log 2>&1 || exit $?
for v in 8 23 20; do timeout -k 10 200 python tools/stamps.py c2 $v > gpurun_out/stamps_v$v.log 2>&1 || exit $?; done
echo done
