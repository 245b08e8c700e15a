#!/bin/bash
# Run the FastTalk service in front of an external inference server (no GPU needed
# by this process): creates .env.remote from the example and starts the WebSocket
# service with the remote provider.
#   VLLM_BASE_URL=http://gpu-node:8000/v1 ./run-remote.sh          # OpenAI-compatible /v1
#   LLM_PROVIDER=ollama OLLAMA_BASE_URL=http://host:11434 ./run-remote.sh
set -euo pipefail
cd "$(dirname "$0")"
[ -f .env.remote ] || cp .env.remote.example .env.remote
# variables given on the command line win over the file (load_env_file keeps them)
source scripts/load_env.sh
load_env_file .env.remote
export COMPUTE_DEVICE=cpu
# the launcher verifies the backend before serving and exits 1 if it is unreachable
exec python main.py websocket "$@"
