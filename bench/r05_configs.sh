#!/bin/bash
# Round-5 measurements at HEAD: driver-config kernel trace, config 5 (agent tools),
# config 2 (one session), AWQ W4A16 at the driver config.
set -o pipefail
mkdir -p gpurun_out
bash bench/gpu_check.sh prof || exit $?
bash gpurun_step.sh \
  "cfg5:400:python bench.py --agent-tools 0.2 --steps 20 --warmup 5" \
  "cfg2:300:python bench.py --sessions 1 --steps 4 --warmup 1" \
  "awq:400:python bench.py --quant awq --steps 20 --warmup 5"
