#!/bin/bash
# decode attention merge batch 16 (was 8): small-batch probe + driver-shape attention + decode test
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "dtest:300:python -u -m pytest tests/test_kernels_gpu.py -q -x -k 'decode_att' --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "sb:200:python bench/attn_small_batch.py" "acfg:300:python bench/attn_cfg.py" "s1:300:python bench.py --sessions 1 --steps 4 --warmup 1" || exit $?
grep "B=1" gpurun_out/sb.log; cat gpurun_out/acfg.log | grep -v amdgpu; python bench/bsum.py gpurun_out/s1.log
