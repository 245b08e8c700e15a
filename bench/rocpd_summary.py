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


def busy(db: str, last_ms: float = 0.0) -> str:
    """GPU busy time (union of kernel intervals) vs wall span, over the whole
    trace or its last ``last_ms`` milliseconds: how much of a step is gaps."""
    c = sqlite3.connect(db)
    iv = sorted(c.execute("select start, end from kernels").fetchall())
    if not iv:
        return "no kernels"
    t1 = max(e for _, e in iv)
    t0 = t1 - last_ms * 1e6 if last_ms else iv[0][0]
    tot, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if e <= t0:
            continue
        s = max(s, t0)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    tot += cur_e - cur_s
    span = t1 - t0
    gaps.sort()
    med = gaps[len(gaps) // 2] / 1e3 if gaps else 0.0
    return (f"window {span / 1e6:.2f} ms: GPU busy {tot / 1e6:.2f} ms ({100 * tot / span:.1f}%), "
            f"{len(gaps)} gaps, median gap {med:.2f} us, gaps > 50 us: "
            f"{sum(g for g in gaps if g > 50e3) / 1e6:.2f} ms")


def gaps_by_kernel(db: str, last_ms: float, top: int = 15) -> str:
    """Idle time before each kernel (previous kernel's end -> this start) over
    the last ``last_ms`` ms, summed per kernel name: where a step's gaps sit."""
    c = sqlite3.connect(db)
    rows = sorted(c.execute("select start, end, name from kernels").fetchall())
    t1 = max(e for _, e, _ in rows)
    t0 = t1 - last_ms * 1e6
    agg, prev_e = {}, None
    for s, e, n in rows:
        if prev_e is not None and s >= t0:
            g = max(0, s - prev_e)
            a = agg.setdefault(n[:90], [0, 0])
            a[0] += g
            a[1] += 1
        prev_e = e if prev_e is None else max(prev_e, e)
    out = [f"{'gap_us':>10} {'n':>6} {'avg':>7}  next kernel"]
    for n, (g, k) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        out.append(f"{g / 1e3:10.0f} {k:6d} {g / 1e3 / k:7.2f}  {n}")
    return "\n".join(out)


def timeline(db: str, last_ms: float, span_ms: float = 30.0, min_gap_us: float = 5.0) -> str:
    """Dispatch sequence of a ``span_ms`` window starting ``last_ms`` before the end:
    every dispatch preceded by an idle gap >= min_gap_us, with its predecessor, so
    a step's bubbles can be placed (what ran before and after each)."""
    c = sqlite3.connect(db)
    rows = sorted(c.execute("select start, end, name from kernels").fetchall())
    t1 = max(e for _, e, _ in rows)
    t0 = t1 - last_ms * 1e6
    out = [f"timeline {span_ms:.0f} ms from t-{last_ms:.0f} ms: gaps >= {min_gap_us:.0f} us"]
    prev = None
    for s, e, n in rows:
        if s < t0:
            prev = (s, e, n)
            continue
        if s > t0 + span_ms * 1e6:
            break
        if prev is not None and (s - prev[1]) / 1e3 >= min_gap_us:
            out.append(f"  t={(prev[0] - t0) / 1e3:9.1f} us  {(prev[1] - prev[0]) / 1e3:7.1f} us  {prev[2][:70]}")
            out.append(f"      gap {(s - prev[1]) / 1e3:8.1f} us -> {(e - s) / 1e3:7.1f} us  {n[:70]}")
        prev = (s, e, n)
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--per-step", type=int, default=0)
    ap.add_argument("--busy-last-ms", type=float, default=-1,
                    help="also report GPU busy vs wall over the last N ms (0: whole trace)")
    a = ap.parse_args()
    print(summarize(a.db, a.top, a.per_step))
    if a.busy_last_ms >= 0:
        print(busy(a.db, a.busy_last_ms))
        if a.busy_last_ms > 0:
            print(gaps_by_kernel(a.db, a.busy_last_ms))
            print(timeline(a.db, a.busy_last_ms / 2))
