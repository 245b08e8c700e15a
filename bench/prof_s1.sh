# Per-kernel profile of single-session decode (bf16 and W4A16) under rocprofv3:
# writes gpurun_out/prof_s1_{bf16,w4}.txt (summary + GPU busy fraction).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SESS=${SESS:-1}
for q in ${QUANTS:-bf16 w4}; do
  if [ $q = w4 ]; then QA="--quant w4"; else QA=""; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s${SESS}_$q -o run -- python3 bench.py $QA --sessions $SESS --steps ${STEPS:-1} --warmup 1 > gpurun_out/prof_s${SESS}_$q.log 2>&1 || exit $?
  db=$(find gpurun_out/prof_s${SESS}_$q -name "*.db" | head -n 1)
  python3 bench/rocpd_summary.py $db --top 30 --busy-last-ms 200 > gpurun_out/prof_s${SESS}_$q.txt || exit $?
  rm -rf gpurun_out/prof_s${SESS}_$q
done
