S="python bench.py --agent-tools 0.2 --steps 20 --warmup 5"
bash gpurun_step.sh "c5A1:400:ENGINE_MIXED_CHAIN=0 $S" "c5B1:400:ENGINE_MIXED_CHAIN=1 $S" "c5A2:400:ENGINE_MIXED_CHAIN=0 $S" "c5B2:400:ENGINE_MIXED_CHAIN=1 $S"
