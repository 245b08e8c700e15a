#!/bin/bash
# PMC passes over W4A16 decode GEMM configs: bench/w4_pmc2.sh <tag> <proj> <nt,splits,xr> [...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/w4pmc2
while [ $# -ge 3 ]; do
  T=$1; P=$2; C=$3; shift 3
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d $R/gpurun_out/w4pmc2/${T}a -o run -- python3 $R/bench/w4_pmc.py --proj $P --cfg $C > $R/gpurun_out/w4pmc2/${T}a.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace -d $R/gpurun_out/w4pmc2/${T}b -o run -- python3 $R/bench/w4_pmc.py --proj $P --cfg $C > $R/gpurun_out/w4pmc2/${T}b.log 2>&1 || exit $?
  for d in a b; do python3 $R/bench/pmc_summary.py $(find $R/gpurun_out/w4pmc2/${T}$d -name "*.db") --match=w4; rm -rf $R/gpurun_out/w4pmc2/${T}$d; done
done
