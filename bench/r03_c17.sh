#!/bin/bash
# 8-wave xr for o/down at 33-64 rows: kernel + engine tests, then same-box bench A/B (A = FT_XR8=0)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "xrtest:400:python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/distributed/test_tp_share_gpu.py -q -x -k 'skinny or xr or llama3_shape or tp_share or graph_decode' --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
AENV="FT_XR8=0" BENV="" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
