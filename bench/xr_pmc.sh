#!/bin/bash
# PMC passes over the decode xr GEMM (gate_up) and the prefill attention
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/xrpmc
P=${1:-gu}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/xrpmc/a -o run -- python3 $R/bench/xr_pmc.py --proj $P > $R/gpurun_out/xrpmc/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/xrpmc/b -o run -- python3 $R/bench/xr_pmc.py --proj $P > $R/gpurun_out/xrpmc/b.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM --kernel-trace -d $R/gpurun_out/xrpmc/c -o run -- python3 $R/bench/xr_pmc.py --proj $P > $R/gpurun_out/xrpmc/c.log 2>&1 || exit $?
for d in a b c; do python3 $R/bench/pmc_summary.py $(find $R/gpurun_out/xrpmc/$d -name "*.db") --match=skinny; done
