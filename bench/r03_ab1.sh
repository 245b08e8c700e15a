#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "tpshare:600:python -u -m pytest tests/distributed/test_tp_share_gpu.py tests/test_kernels_gpu.py -q -k \"tp_share or prefill or decode_att\" --timeout 300 --timeout-method thread -p no:cacheprovider" "pf:300:python bench/prefill_probe.py --cases 5:107:3000,10:100:3000,4:128:3000,1:512:3000,1:2048:0" || exit $?
bash bench/ab_trees.sh "python bench/attn_cfg.py" 2 > gpurun_out/ab_attn.txt 2>&1 || exit $?
mkdir -p gpurun_out/abattn && mv gpurun_out/ab_[AB]*.log gpurun_out/abattn/
bash bench/ab_trees.sh "python bench/mixed_probe.py --reps 3" 1 > gpurun_out/ab_mixed.txt 2>&1 || exit $?
mkdir -p gpurun_out/abmixed && mv gpurun_out/ab_[AB]*.log gpurun_out/abmixed/
bash bench/ab_trees.sh "python bench.py --gpus 1 --steps 20 --warmup 5" 2 > gpurun_out/ab_bench.txt 2>&1 || exit $?
cat gpurun_out/ab_attn.txt gpurun_out/ab_mixed.txt gpurun_out/ab_bench.txt
