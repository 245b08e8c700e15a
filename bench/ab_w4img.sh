S="python bench.py --quant awq --steps 20 --warmup 5"
bash gpurun_step.sh "wt:600:timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -q -x -k 'w4 or awq or quant' --timeout 120 --timeout-method thread" "wA1:400:FT_W4_PREFILL_IMAGE=0 $S" "wB1:400:$S" "wA2:400:FT_W4_PREFILL_IMAGE=0 $S" "wB2:400:$S"
