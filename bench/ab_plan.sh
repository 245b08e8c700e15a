#!/bin/bash
# Engine A/B of a PACKED_PLAN overlay (A = the overlay, B = the plan in llama.py),
# driver-style bench.py runs, interleaved A B A B.
PLAN=${PLAN:-'{"qkv": {"64": [2, -4, 8]}, "o": {"64": [2, -4, 8]}, "gu": {"64": [2, -4, 2]}, "down": {"64": [4, -3, 4]}, "lm": {"64": [2, -4, 1]}}'}
STEPS=${STEPS:-10}
bash gpurun_step.sh \
 "abA1:300:FT_PACKED_PLAN='$PLAN' python bench.py --steps $STEPS --warmup 3" \
 "abB1:300:python bench.py --steps $STEPS --warmup 3" \
 "abA2:300:FT_PACKED_PLAN='$PLAN' python bench.py --steps $STEPS --warmup 3" \
 "abB2:300:python bench.py --steps $STEPS --warmup 3"
