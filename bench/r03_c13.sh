#!/bin/bash
# refresh the secondary configs at round-3 HEAD: AWQ at the driver config, config 5 (agent tools), config 2 (1 session)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "awq:400:python bench.py --quant awq --steps 20 --warmup 5" \
  "tools:400:python bench.py --agent-tools 0.2 --steps 20 --warmup 5" \
  "s1:300:python bench.py --sessions 1 --steps 4 --warmup 1" || exit $?
for f in awq tools s1; do python bench/bsum.py gpurun_out/$f.log; done
