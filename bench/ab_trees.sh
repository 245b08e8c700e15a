#!/bin/bash
# Same-box A/B of two source trees: A = ab_old/ (a git worktree at the baseline
# revision, built in place), B = this tree.  usage: bench/ab_trees.sh "<cmd>" [reps]
# Each arm runs from its own tree root; output -> gpurun_out/ab_{A,B}{i}.log
cd "$(dirname "$0")/.."
R=$(pwd)
CMD="$1"; REPS=${2:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq 1 $REPS); do
  for arm in A B; do
    if [ $arm = A ]; then d=$R/ab_old; else d=$R; fi
    (cd $d && timeout -k 10 600 bash -c "$CMD") > gpurun_out/ab_$arm$i.log 2>&1
    rc=$?
    echo "== $arm$i rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$arm$i.log | tail -4
    if [ $rc -ge 2 ]; then exit $rc; fi
  done
done
