#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh \
  "ktests:600:python -u -m pytest tests/test_kernels_gpu.py tests/distributed/test_tp_share_gpu.py -q -k 'w4 or prefill or decode_att or tp_share' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "w4xr:400:python bench/w4xr_sweep.py" \
  "pf:300:python bench/prefill_probe.py --cases 5:107:3000,10:100:3000,4:128:3000,1:512:3000,1:2048:0" \
  "abattn:400:bash bench/ab_trees.sh 'python bench/attn_cfg.py' 2"
