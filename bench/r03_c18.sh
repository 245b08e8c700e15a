#!/bin/bash
# prefill split plan: per-item overhead constant sweep (FT_PREFILL_ITEM_TILES)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
C="5:107:3000,10:100:3000,4:128:3000,3:150:4000,1:512:3000,6:80:2500,8:60:3500,2:200:1500"
./gpurun_step.sh "it05:200:FT_PREFILL_ITEM_TILES=0.5 python bench/prefill_probe.py --cases $C" \
  "it1:200:FT_PREFILL_ITEM_TILES=1 python bench/prefill_probe.py --cases $C" \
  "it2:200:FT_PREFILL_ITEM_TILES=2 python bench/prefill_probe.py --cases $C" \
  "it4:200:FT_PREFILL_ITEM_TILES=4 python bench/prefill_probe.py --cases $C" \
  "it1b:200:FT_PREFILL_ITEM_TILES=1 python bench/prefill_probe.py --cases $C" || exit $?
for f in it05 it1 it2 it4 it1b; do echo "== $f"; grep '^{' gpurun_out/$f.log | python3 -c "import sys,json; print('  '.join(f\"{d['seqs']}x{d['new']}/{d['ctx']}: {d['us']}us w{d['wgs']}\" for d in map(json.loads, sys.stdin)))"; done
