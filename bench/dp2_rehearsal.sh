#!/bin/bash
# The driver's multi-GPU launch form with both ranks time-sharing ONE MI355X
# (FT_BENCH_SHARED_GPU=1): a topology / code-path check, not a scaling number.
mkdir -p gpurun_out
FT_BENCH_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  > gpurun_out/dp2_rehearsal.log 2>&1; rc=$?
grep '^{"metric"' gpurun_out/dp2_rehearsal.log; tail -n 3 gpurun_out/dp2_rehearsal.log; exit $rc
