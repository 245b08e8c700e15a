S5="python bench.py --agent-tools 0.2 --steps 20 --warmup 5"
S="python bench.py --steps 20 --warmup 5"
bash gpurun_step.sh "fA1:400:ENGINE_PREFILL_FLOOD=1 $S5" "fB1:400:$S5" "fA2:400:ENGINE_PREFILL_FLOOD=1 $S5" "fB2:400:$S5" "gA:300:ENGINE_PREFILL_FLOOD=1 $S" "gB:300:$S"
