#!/bin/bash
# One GPU call: GPU test suite, then a rocprofv3 kernel trace of the driver's
# headline config (bench.py --steps 20 --warmup 5), summarised per kernel.
# usage: bench/gpu_check.sh [tests] [smoke] [bench] [benchrank] [prof] [prof70]   (default: tests prof)
set -o pipefail
mkdir -p gpurun_out
what="${*:-tests prof}"
for w in $what; do
  case $w in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/gputests.log 2>&1; rc=$?; tail -n 5 gpurun_out/gputests.log
      [ $rc -ne 0 ] && exit $rc ;;
    prof)
      rm -rf /tmp/ftprof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/ftprof -o run -- \
        python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/prof_bench.log 2>&1; rc=$?
      tail -n 3 gpurun_out/prof_bench.log
      [ $rc -ne 0 ] && exit $rc
      db=$(find /tmp/ftprof -name '*.db' | sort | tail -n 1)
      python3 bench/rocpd_summary.py "$db" --top 45 --busy-last-ms 200 > gpurun_out/prof_summary.txt 2>&1
      find /tmp/ftprof -name '*stats*.csv' -exec cp {} gpurun_out/ \;
      sed -n 1,30p gpurun_out/prof_summary.txt ;;
    bench)
      timeout -k 10 600 python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench.log 2>&1; rc=$?
      tail -n 3 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc ;;
    benchrank)   # same config, engine socket served by the rank itself (no front door)
      timeout -k 10 600 python3 bench.py --serve rank --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_rank.log 2>&1; rc=$?
      tail -n 3 gpurun_out/bench_rank.log; [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -n 3 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc ;;
    prof70)      # Llama-3-70B TP=1 at 50 sessions, per-kernel table over the last 20 s
      rm -rf /tmp/ftprof70
      timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/ftprof70 -o run -- \
        python3 bench.py --model llama3-70b --sessions 50 --steps 3 --warmup 1 > gpurun_out/prof70_bench.log 2>&1; rc=$?
      tail -n 3 gpurun_out/prof70_bench.log
      [ $rc -ne 0 ] && exit $rc
      db=$(find /tmp/ftprof70 -name '*.db' | sort | tail -n 1)
      python3 bench/rocpd_summary.py "$db" --top 40 --busy-last-ms 20000 > gpurun_out/prof70_summary.txt 2>&1
      sed -n 1,20p gpurun_out/prof70_summary.txt ;;
  esac
done
exit 0
