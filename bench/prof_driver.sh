# Kernel trace of the driver-config bench (bench.py --steps 20 --warmup 5) under
# rocprofv3: gpurun_out/prof_driver.txt = per-kernel table + GPU busy / gaps over
# the last BUSY_MS ms (default 15 s, all inside the timed turns).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_drv -o run -- python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/prof_driver.log 2>&1 || exit $?
db=$(find gpurun_out/prof_drv -name "*.db" | head -n 1)
python3 bench/rocpd_summary.py $db --top 40 --busy-last-ms ${BUSY_MS:-15000} > gpurun_out/prof_driver.txt || exit $?
rm -rf gpurun_out/prof_drv
