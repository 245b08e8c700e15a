#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh \
  "agent:600:python bench.py --gpus 1 --steps 20 --warmup 5 --agent-tools 0.2" \
  "s1:400:python bench.py --sessions 1 --steps 4 --warmup 1 --gen 256" \
  "profdrv:700:bash bench/prof_driver.sh"
