#!/bin/bash
# rocprofv3 kernel trace of config 5 (agent tools 20%) at HEAD, summarised per kernel
# with the GPU-busy share of the timed window
set -o pipefail
mkdir -p gpurun_out
rm -rf /tmp/ftprof5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/ftprof5 -o run -- \
  python3 bench.py --agent-tools 0.2 --steps 20 --warmup 5 > gpurun_out/prof5_bench.log 2>&1 || exit $?
tail -n 2 gpurun_out/prof5_bench.log
db=$(find /tmp/ftprof5 -name '*.db' | sort | tail -n 1)
python3 bench/rocpd_summary.py "$db" --top 45 --busy-last-ms 15000 > gpurun_out/prof5_summary.txt 2>&1
sed -n 1,12p gpurun_out/prof5_summary.txt
