#!/bin/bash
# Engine A/B of an environment setting: A = "$AENV", B = "$BENV" (default empty),
# driver-style bench.py runs interleaved A B A B.
STEPS=${STEPS:-10}
bash gpurun_step.sh \
 "abA1:300:$AENV python bench.py --steps $STEPS --warmup ${WARMUP:-3}" \
 "abB1:300:$BENV python bench.py --steps $STEPS --warmup ${WARMUP:-3}" \
 "abA2:300:$AENV python bench.py --steps $STEPS --warmup ${WARMUP:-3}" \
 "abB2:300:$BENV python bench.py --steps $STEPS --warmup ${WARMUP:-3}"
