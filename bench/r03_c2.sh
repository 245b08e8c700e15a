#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh \
  "w4e2e:600:python -u -m pytest tests/test_engine_gpu.py -q -k 'w4' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "awq:600:python bench.py --gpus 1 --steps 20 --warmup 5 --quant awq" \
  "abbench:1000:bash bench/ab_trees.sh 'python bench.py --gpus 1 --steps 20 --warmup 5' 2"
