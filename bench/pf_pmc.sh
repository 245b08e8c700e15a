#!/bin/bash
# PMC passes over the prefill attention probe (one counter group per run, kernel trace only)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CASES=${1:-10:100:3000}
mkdir -p $R/gpurun_out/pfpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/pfpmc/a -o run -- python3 $R/bench/prefill_probe.py --cases $CASES > $R/gpurun_out/pfpmc/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pfpmc/b -o run -- python3 $R/bench/prefill_probe.py --cases $CASES > $R/gpurun_out/pfpmc/b.log 2>&1 || exit $?
for d in a b; do python3 $R/bench/pmc_summary.py $(find $R/gpurun_out/pfpmc/$d -name "*.db") --match=prefill; done
