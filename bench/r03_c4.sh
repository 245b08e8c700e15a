#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh \
  "sktest:400:python -u -m pytest tests/test_kernels_gpu.py -q -k 'stream_k' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "skprobe:300:python bench/sk_probe.py" \
  "e2e:600:python -u -m pytest tests/test_engine_gpu.py -q -k 'shape_decode or graph_decode or logits_match' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench:400:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "benchoff:400:FT_SK=0 python bench.py --gpus 1 --steps 20 --warmup 5"
