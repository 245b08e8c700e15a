S5="python bench.py --agent-tools 0.2 --steps 20 --warmup 5"
S="python bench.py --steps 20 --warmup 5"
bash gpurun_step.sh "bA1:400:FT_STEP_TRACE=\$PWD/gpurun_out/tA1.json $S5" "bB1:400:FT_PG_BLAS_ROWS=0 FT_STEP_TRACE=\$PWD/gpurun_out/tB1.json $S5" "bA2:400:$S5" "bB2:400:FT_PG_BLAS_ROWS=0 $S5" "dA:300:$S" "dB:300:FT_PG_BLAS_ROWS=0 $S"
