S="python bench.py --steps 20 --warmup 5"
bash gpurun_step.sh "sc0:300:$S" "sc640:300:ENGINE_PREFILL_CHUNK=640 $S" "sc384:300:ENGINE_PREFILL_CHUNK=384 $S" "scm90:300:ENGINE_MIXED_CHAIN_AT=0.9 $S" "scm60:300:ENGINE_MIXED_CHAIN_AT=0.6 $S" "sc0b:300:$S"
