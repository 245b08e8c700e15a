#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
./gpurun_step.sh "xrpmc:300:bash bench/xr_pmc.sh gu" "pfpmc:300:bash bench/pf_pmc.sh 10:100:3000"
