#!/bin/bash
# 8-wave xr for o/down at 33-64 rows: kernel tests, engine tests with FT_XR8=1, then same-box bench A/B (B = FT_XR8=1)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "xrtest:300:python -u -m pytest tests/test_kernels_gpu.py -q -x -k 'skinny or xr' --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "xr8eng:500:FT_XR8=1 python -u -m pytest tests/test_engine_gpu.py tests/distributed/test_tp_share_gpu.py -q -x -k 'llama3_shape or tp_share or graph_decode or pipelined' --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
AENV="" BENV="FT_XR8=1" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
