S="python bench.py --steps 20 --warmup 5"
C="ENGINE_PREFILL_CHUNK=384 ENGINE_MIXED_CHAIN_AT=0.6"
bash gpurun_step.sh "cfA1:300:$S" "cfB1:300:$C $S" "cfA2:300:$S" "cfB2:300:$C $S" "cfC1:300:ENGINE_MIXED_CHAIN_AT=0.6 $S" "cfC2:300:ENGINE_MIXED_CHAIN_AT=0.6 $S"
