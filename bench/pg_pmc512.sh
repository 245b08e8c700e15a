#!/bin/bash
# PMC passes over packed_gemm cfg 0 (gate_up, 512 rows, SiLU off) vs hipBLASLt.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc512
for arm in "pg:--cfg 0" "blas:--blas"; do
  name="${arm%%:*}"; args="${arm#*:}"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/pmc512/$name-a -o run -- python3 $R/bench/pg_pmc.py --m 512 $args > $R/gpurun_out/pmc512/$name-a.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY --kernel-trace -d $R/gpurun_out/pmc512/$name-b -o run -- python3 $R/bench/pg_pmc.py --m 512 $args > $R/gpurun_out/pmc512/$name-b.log 2>&1 || exit $?
  for d in a b; do python3 $R/bench/pmc_summary.py $(find $R/gpurun_out/pmc512/$name-$d -name "*.db") ; done
done
echo pmc done
