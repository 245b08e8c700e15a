#!/bin/bash
# (1) mixed-ahead without JIT vs both off; (2) row-major copies A/B (+ logits test at 300 rows)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "lgtests:400:python -u -m pytest tests/test_engine_gpu.py -q -x -k 'logits_match_cpu or single_weight_image' --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
AENV="ENGINE_MIXED_AHEAD=0 ENGINE_JIT_TOPUP=0" BENV="ENGINE_JIT_TOPUP=0" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
mkdir -p gpurun_out/ab_mx && cp gpurun_out/ab[AB][12].log gpurun_out/ab_mx/
AENV="FT_ROWMAJOR_COPIES=0 ENGINE_MIXED_AHEAD=0 ENGINE_JIT_TOPUP=0" BENV="ENGINE_MIXED_AHEAD=0 ENGINE_JIT_TOPUP=0" STEPS=20 WARMUP=5 bash bench/ab_env.sh || exit $?
mkdir -p gpurun_out/ab_rm && cp gpurun_out/ab[AB][12].log gpurun_out/ab_rm/
for d in ab_mx ab_rm; do echo "== $d"; python bench/bsum.py gpurun_out/$d/abA1.log gpurun_out/$d/abB1.log gpurun_out/$d/abA2.log gpurun_out/$d/abB2.log; done
for f in gpurun_out/ab_mx/abB1.log gpurun_out/ab_mx/abB2.log; do grep -o '"engine_steps": {[^}]*}' $f; done
