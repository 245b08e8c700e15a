#!/bin/bash
# Run FastTalk on MI355X GPUs (bare metal): creates .env from the example,
# builds the gfx950 kernels + C++ runtime in-tree, starts the WebSocket service.
#   ./run-rocm.sh                      # 1 GPU, Llama-3.1-8B (random weights)
#   ENGINE_DP_SIZE=8 ./run-rocm.sh     # 8 replicas, session-affine routing
#   ENGINE_TP_SIZE=8 ENGINE_MODEL=llama3-70b ./run-rocm.sh
set -euo pipefail
cd "$(dirname "$0")"
[ -f .env ] || cp .env.example .env
source scripts/load_env.sh
load_env_file .env
export COMPUTE_DEVICE=${COMPUTE_DEVICE:-rocm} HSA_ENABLE_IPC_MODE_LEGACY=0 PYTORCH_ROCM_ARCH=gfx950
python -m fasttalk_llm_microservice_amd.ops.build
exec python main.py websocket "$@"
