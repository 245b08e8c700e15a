#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "sb2:200:python bench/attn_small_batch.py" "sb3:200:FT_DECODE_RING=3 python bench/attn_small_batch.py" "sb4:200:FT_DECODE_RING=4 python bench/attn_small_batch.py" "sbw2:200:FT_DECODE_WPC=2 python bench/attn_small_batch.py" || exit $?
for f in sb2 sb3 sb4 sbw2; do echo "== $f"; grep "B=1" gpurun_out/$f.log; done
