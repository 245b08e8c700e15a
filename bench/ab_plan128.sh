S="python bench.py --steps 20 --warmup 5"
bash gpurun_step.sh "pA1:300:FT_PG_PLAN=r4 $S" "pB1:300:$S" "pA2:300:FT_PG_PLAN=r4 $S" "pB2:300:$S"
