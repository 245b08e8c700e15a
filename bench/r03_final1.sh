#!/bin/bash
# full GPU suite + smoke + rocprof kernel table of the driver config + one plain bench run
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "gpufull:1000:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench:400:python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
bash bench/prof_driver.sh > gpurun_out/profdrv.log 2>&1 || exit $?
tail -3 gpurun_out/profdrv.log
