#!/bin/bash
# Container entrypoint: build the native extensions if the image was built
# without them (e.g. a bind-mounted source tree), then run the service CLI.
set -e
if ! python -c "import fasttalk_llm_microservice_amd._C, fasttalk_llm_microservice_amd._rt" 2>/dev/null; then
  echo "[entrypoint] building gfx950 kernels + runtime"
  python -m fasttalk_llm_microservice_amd.ops.build
fi
exec python main.py "$@"
