"""Per-kernel PMC counter means from rocprofv3 rocpd databases.
python bench/pmc_summary.py <run_results.db>... [--match substring]"""
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "")
for path in args:
    db = sqlite3.connect(path)
    rows = db.execute("select kernel_name, dispatch_id, counter_name, value, duration "
                      "from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for k, d, c, v, du in rows:
        if match and match not in k:
            continue
        per[k][c].append(v)
        dur[k][d] = du
    print(f"== {path}")
    for k, cs in per.items():
        if len(dur[k]) < 3:
            continue
        ds = sorted(dur[k].values())
        print(f"  {k[:90]}  dispatches {len(ds)}  median {ds[len(ds) // 2] / 1e3:.1f} us")
        for c, vs in sorted(cs.items()):
            vs = vs[2:] if len(vs) > 4 else vs
            print(f"    {c:28s} {sum(vs) / len(vs):16.0f}")
