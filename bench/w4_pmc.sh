#!/bin/bash
# PMC passes over the W4A16 decode GEMMs (one projection per call; default all four)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/w4pmc
for P in ${@:-gu qkv o down}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/w4pmc/${P}a -o run -- python3 $R/bench/w4_pmc.py --proj $P > $R/gpurun_out/w4pmc/${P}a.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM --kernel-trace -d $R/gpurun_out/w4pmc/${P}c -o run -- python3 $R/bench/w4_pmc.py --proj $P > $R/gpurun_out/w4pmc/${P}c.log 2>&1 || exit $?
  for d in a c; do python3 $R/bench/pmc_summary.py $(find $R/gpurun_out/w4pmc/${P}$d -name "*.db") --match=w4; done
done
