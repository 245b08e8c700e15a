#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh \
  "w4test:600:python -u -m pytest tests/test_engine_gpu.py -x -q -k 'shape_decode and w4' --timeout 300 --timeout-method thread" \
  "pfpmc:400:bash bench/pf_pmc.sh 10:100:3000" \
  "profs1:450:bash bench/prof_s1.sh" \
  "awq:600:python bench.py --gpus 1 --steps 20 --warmup 5 --quant awq"
