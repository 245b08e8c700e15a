#!/bin/bash
# PMC passes over the engine's decode hot kernels (paged decode attention, skinny_xr GEMMs, row
# kernels): engine_bench in eager mode (kernels replayed inside hipGraphs are not counter-profiled),
# 50 sequences x 3000-token prompts, one counter group per run, kernel trace only.
# usage (GPU box): bash bench/decode_pmc.sh ; summaries in gpurun_out/decpmc/*.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/decpmc
mkdir -p $O
CMD="python3 $R/bench/engine_bench.py --seqs 50 --prompt 3000 --gen 24 --rounds 1 --eager"
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace -d $O/a -o run -- $CMD > $O/a.log 2>&1 || exit $?
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $O/b -o run -- $CMD > $O/b.log 2>&1 || exit $?
for d in a b; do
  python3 $R/bench/pmc_summary.py $(find $O/$d -name "*.db") --match=ft:: > $O/$d.txt || exit $?
done
rm -rf $O/a $O/b   # the databases exceed what gpurun copies back; the summaries stay
