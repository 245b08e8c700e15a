# Kernel trace of the single-session bench (BASELINE config 2, Llama-3-8B, one WS
# session): gpurun_out/prof_s1.txt = per-kernel table with time per decode step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_s1 -o run -- python3 bench.py --sessions 1 --steps ${STEPS:-4} --warmup ${WARMUP:-1} --gen 256 > gpurun_out/prof_s1.log 2>&1 || exit $?
db=$(find gpurun_out/prof_s1 -name "*.db" | head -n 1)
python3 bench/rocpd_summary.py $db --top 30 --per-step $(( ${STEPS:-4} * 256 + ${WARMUP:-1} * 256 )) --busy-last-ms ${BUSY_MS:-2000} > gpurun_out/prof_s1.txt || exit $?
rm -rf gpurun_out/prof_s1
