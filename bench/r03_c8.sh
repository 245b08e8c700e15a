#!/bin/bash
# mixed-ahead + JIT top-up: GPU engine tests, then same-box bench A/B (A = both off, B = default on)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "etests:500:python -u -m pytest tests/test_engine_gpu.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
AENV="ENGINE_MIXED_AHEAD=0 ENGINE_JIT_TOPUP=0" BENV="" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
python bench/bsum.py gpurun_out/abA1.log gpurun_out/abB1.log gpurun_out/abA2.log gpurun_out/abB2.log
for f in gpurun_out/abA1.log gpurun_out/abB1.log; do grep -o '"engine_steps": {[^}]*}' $f; grep -o '"engine_runner": {[^}]*}' $f; done
