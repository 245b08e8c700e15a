#!/bin/bash
# pipelined-decode shrink: GPU test + same-box engine A/B (A = drain on stop, B = shrink)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "pipetest:300:python -u -m pytest tests/test_engine_gpu.py -q -k 'pipelined or many_sequences' --timeout 240 --timeout-method thread -p no:cacheprovider" || exit $?
AENV="ENGINE_PIPELINE_SHRINK=0" BENV="" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
for f in gpurun_out/abA1.log gpurun_out/abB1.log; do grep -o '"engine_steps": {[^}]*}' $f; done
