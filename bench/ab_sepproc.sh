S="python bench.py --steps 20 --warmup 5"
bash gpurun_step.sh "spA1:300:$S" "spB1:300:ENGINE_SEPARATE_PROCESS=1 $S" "spA2:300:$S" "spB2:300:ENGINE_SEPARATE_PROCESS=1 $S"
