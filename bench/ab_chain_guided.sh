S5="python bench.py --agent-tools 0.2 --steps 20 --warmup 5"
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -q -x -k "guided or tool or json or pipelin" --timeout 200 --timeout-method thread > gpurun_out/cg_tests.log 2>&1 || exit 1
bash gpurun_step.sh "cgA1:400:ENGINE_MIXED_CHAIN_GUIDED=0 $S5" "cgB1:400:$S5" "cgA2:400:ENGINE_MIXED_CHAIN_GUIDED=0 $S5" "cgB2:400:$S5"
