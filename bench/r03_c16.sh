#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "xrtest:300:python -u -m pytest tests/test_kernels_gpu.py -q -x -k 'xr or skinny' --timeout 240 --timeout-method thread -p no:cacheprovider" "xr8:400:python bench/xr8_sweep.py" || exit $?
grep -v amdgpu gpurun_out/xr8.log
