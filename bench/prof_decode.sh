# Kernel trace of steady 50-sequence decode at ~3k context (engine_bench, no WS):
# gpurun_out/prof_decode.txt = per-kernel table + GPU busy and gaps over the last 300 ms.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/prof_dec -o run -- python3 bench/engine_bench.py --seqs ${SEQS:-50} --prompt ${PROMPT:-3000} --gen ${GEN:-160} --rounds 1 > gpurun_out/prof_decode.log 2>&1 || exit $?
db=$(find gpurun_out/prof_dec -name "*.db" | head -n 1)
python3 bench/rocpd_summary.py $db --top 30 --busy-last-ms 300 > gpurun_out/prof_decode.txt || exit $?
rm -rf gpurun_out/prof_dec
