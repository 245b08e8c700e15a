#!/bin/bash
# PMC passes over the decode hot kernels with fp8 vs bf16 KV caches (decode attention's
# HBM bytes, VALU / MFMA work and waits): engine_bench in eager mode, 50 sequences x
# 3000-token prompts, one counter group per run, kernel trace only.
# usage (GPU box): bash bench/decode_pmc_fp8.sh ; summaries in gpurun_out/decpmc8/*.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/decpmc8
mkdir -p $O
for kv in fp8 auto; do
  CMD="python3 $R/bench/engine_bench.py --seqs 50 --prompt 3000 --gen 24 --rounds 1 --eager --kv-cache-dtype $kv"
  timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-trace -d $O/a_$kv -o run -- $CMD > $O/a_$kv.log 2>&1 || exit $?
  timeout -s KILL 170 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/b_$kv -o run -- $CMD > $O/b_$kv.log 2>&1 || exit $?
  for d in a_$kv b_$kv; do
    python3 $R/bench/pmc_summary.py $(find $O/$d -name "*.db") --match=paged_decode > $O/$d.txt || exit $?
  done
  rm -rf $O/a_$kv $O/b_$kv
done
