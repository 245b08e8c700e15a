#!/bin/bash
# Round-5 final HEAD numbers for the secondary configs: config 5 (agent tools 20%),
# config 2 (one session), AWQ W4A16 at the driver config.
mkdir -p gpurun_out
bash gpurun_step.sh \
  "fcfg5:400:python bench.py --agent-tools 0.2 --steps 20 --warmup 5" \
  "fcfg2:300:python bench.py --sessions 1 --steps 4 --warmup 1" \
  "fawq:400:python bench.py --quant awq --steps 20 --warmup 5"
