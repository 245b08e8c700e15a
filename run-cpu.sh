#!/bin/bash
# Run FastTalk on the CPU backend (fp32 reference ops; plumbing / development).
set -euo pipefail
cd "$(dirname "$0")"
[ -f .env ] || cp .env.example .env
source scripts/load_env.sh
load_env_file .env
export COMPUTE_DEVICE=cpu ENGINE_DEVICE=cpu ENGINE_MODEL=${CPU_MODEL:-llama3.2-1b}
export ENGINE_MAX_NUM_SEQS=${ENGINE_MAX_NUM_SEQS:-8} ENGINE_MAX_MODEL_LEN=${ENGINE_MAX_MODEL_LEN:-2048}
python -m fasttalk_llm_microservice_amd.ops.build --only runtime
exec python main.py websocket "$@"
