#!/bin/bash
PLAN='{"qkv": {"64": [2, -4, 8], "32": [2, -4, 8]}, "o": {"64": [2, -4, 8]}}'
bash gpurun_step.sh \
 "abA1:300:python bench.py --steps 10 --warmup 3" \
 "abB1:300:FT_PACKED_PLAN='$PLAN' python bench.py --steps 10 --warmup 3" \
 "abA2:300:python bench.py --steps 10 --warmup 3" \
 "abB2:300:FT_PACKED_PLAN='$PLAN' python bench.py --steps 10 --warmup 3"
