#!/bin/bash
# end-of-session check: full GPU suite + smoke + driver bench at HEAD
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "gpufull:1000:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench:400:python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
python bench/bsum.py gpurun_out/bench.log
