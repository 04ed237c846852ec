set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
HDFS_CRC32C_KVARIANT=17 timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests17.log 2>&1; rc=$?; echo "tests17 rc=$rc"; tail -3 gpurun_out/tests17.log
if [ $rc -gt 1 ]; then exit $rc; fi
HDFS_CRC32C_KVARIANT=18 timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests18.log 2>&1; rc=$?; echo "tests18 rc=$rc"; tail -3 gpurun_out/tests18.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py --config c2 --variants 0,17,18,19,20 > gpurun_out/kbench.log 2>&1 || exit $?
PV=0,17,18 bash tools/power_probe.sh
