"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd SQLite, the ROCm 7
default output) into a per-kernel table: total/avg time, calls, share.

python bench/rocpd_summary.py gpurun_out/prof/run_results.db [--top 40] [--per-step N]
"""
from __future__ import annotations

import argparse
import sqlite3


def summarize(db: str, top: int = 40, per_step: int = 0) -> str:
    c = sqlite3.connect(db)
    tot = c.execute("select sum(end-start) from kernels").fetchone()[0] or 1
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start) from kernels "
                     "group by name order by sum(end-start) desc limit ?", (top,)).fetchall()
    out = [f"total kernel time: {tot / 1e6:.2f} ms over "
           f"{c.execute('select count(*) from kernels').fetchone()[0]} dispatches",
           f"{'total_us':>12} {'share':>6} {'calls':>7} {'avg_us':>9}"
           + (f" {'us/step':>9}" if per_step else "") + "  kernel"]
    for name, n, s, a in rows:
        line = f"{s / 1e3:12.0f} {100 * s / tot:5.1f}% {n:7d} {a / 1e3:9.2f}"
        if per_step:
            line += f" {s / 1e3 / per_step:9.1f}"
        out.append(line + "  " + name[:120])
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--per-step", type=int, default=0)
    a = ap.parse_args()
    print(summarize(a.db, a.top, a.per_step))
