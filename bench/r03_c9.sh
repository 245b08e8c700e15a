#!/bin/bash
# resident row-major copies (hipBLASLt for qkv/o/gate_up at >= 257 rows): logits test, mixed-step probe + bench A/B
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "lgtests:400:python -u -m pytest tests/test_engine_gpu.py -q -x -k 'logits_match_cpu or chunked or prefix_cache' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "mxA:300:FT_ROWMAJOR_COPIES=0 python bench/mixed_probe.py --reps 3" \
  "mxB:300:python bench/mixed_probe.py --reps 3" || exit $?
AENV="FT_ROWMAJOR_COPIES=0" BENV="" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
