#!/bin/bash
# round-3 re-baseline at HEAD: GPU tests, driver-config bench, mixed-step and prefill probes
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh \
  "gputests:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench:600:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "mixed:300:python bench/mixed_probe.py --reps 4" \
  "prefill:300:python bench/prefill_probe.py --cases 5:107:3000,10:100:3000,4:128:3000,1:512:3000,1:2048:0"
