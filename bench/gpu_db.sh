set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_block_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/db_test.log 2>&1; rc=$?
tail -n 3 gpurun_out/db_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench/block_probe.py "$@" > gpurun_out/db_probe.log 2>&1; rc=$?
cat gpurun_out/db_probe.log
[ $rc -ne 0 ] && exit $rc
FT_DB_PREFETCH=0 timeout -k 10 300 python -u bench/block_probe.py "$@" > gpurun_out/db_probe_nopf.log 2>&1; rc=$?
cat gpurun_out/db_probe_nopf.log
exit $rc
