#!/bin/bash
# PMC passes over the packed GEMM vs hipBLASLt (one counter group per run).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
for arm in "pg:--cfg 0" "blas:--blas"; do
  name="${arm%%:*}"; args="${arm#*:}"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/pmc/$name-a -o run -- python3 $R/bench/pg_pmc.py $args > $R/gpurun_out/pmc/$name-a.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc/$name-b -o run -- python3 $R/bench/pg_pmc.py $args > $R/gpurun_out/pmc/$name-b.log 2>&1
done
echo pmc done
