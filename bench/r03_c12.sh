#!/bin/bash
# drain-time mixed injection: GPU engine test + same-box bench A/B (A = ENGINE_MIXED_AHEAD=0, B = default)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "mxtest:300:python -u -m pytest tests/test_engine_gpu.py -q -x -k 'mixed_ahead or pipelined' --timeout 240 --timeout-method thread -p no:cacheprovider" || exit $?
AENV="ENGINE_MIXED_AHEAD=0" BENV="" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
for f in gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log; do grep -o '"engine_steps": {[^}]*}' $f; done
