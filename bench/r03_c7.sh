#!/bin/bash
# round-aware prefill split plan: kernel tests + probe A/B (A = round-blind plan, B = new) + mixed step A/B
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
C="5:107:3000,10:100:3000,4:128:3000,3:150:4000,1:512:3000,1:2048:0,6:80:2500"
./gpurun_step.sh "ktests:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k 'prefill or pipelined' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "pfA:200:FT_PREFILL_ROUND_BLIND=1 python bench/prefill_probe.py --cases $C" \
  "pfB:200:python bench/prefill_probe.py --cases $C" \
  "pfA2:200:FT_PREFILL_ROUND_BLIND=1 python bench/prefill_probe.py --cases $C" \
  "pfB2:200:python bench/prefill_probe.py --cases $C" \
  "mxA:300:FT_PREFILL_ROUND_BLIND=1 python bench/mixed_probe.py --reps 3" \
  "mxB:300:python bench/mixed_probe.py --reps 3" || exit $?
AENV="FT_PREFILL_ROUND_BLIND=1" BENV="" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
