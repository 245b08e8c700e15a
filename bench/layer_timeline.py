"""Per-kernel timeline of graph-replayed decode steps from a rocprofv3 kernel
trace (rocpd SQLite): for every kernel position of a decode step (embed, then
per layer qkv -> rope/KV -> attention -> o -> add+norm -> gate_up -> down ->
add+norm, then LM head + sampler) the mean duration and the mean idle gap in
front of it, averaged over the decode steps of the trace.  Shows where a step's
time goes beyond the kernels' own work: launch boundaries, ramp-up, tails.

python bench/layer_timeline.py gpurun_out/prof/run_results.db [--steps 200]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sqlite3
from collections import defaultdict


def _short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("ft::", "")
    return name[:60]


def _load(path: str):
    """(name, start_ns, end_ns) rows in start order from a rocprofv3 output: a
    directory (its first *kernel_trace.csv, else its first .db), a CSV or a rocpd db."""
    if os.path.isdir(path):
        found = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))
        found = found or sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
        if not found:
            raise SystemExit(f"no kernel trace under {path}")
        path = found[0]
    if path.endswith(".csv"):
        with open(path, newline="") as f:
            rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                    for r in csv.DictReader(f)]
        return sorted(rows, key=lambda r: r[1])
    c = sqlite3.connect(path)
    try:
        return c.execute("select name, start, end from kernels order by start").fetchall()
    except sqlite3.Error:
        tabs = [r[0] for r in c.execute("select name from sqlite_master")]
        raise SystemExit(f"no 'kernels' view in {path}; objects: {tabs}")


def _mixed_summary(mixed):
    """Mixed (prefill + decode) steps run eagerly: how much of their span the GPU
    is busy (the rest is the host enqueueing kernels one by one), and where their
    kernel time goes."""
    span = busy = 0.0
    agg = defaultdict(lambda: [0, 0.0])
    for st in mixed:
        span += (st[-1][2] - st[0][1]) / 1e3
        for n, s, e in st:
            busy += (e - s) / 1e3
            agg[n][0] += 1
            agg[n][1] += (e - s) / 1e3
    m = len(mixed)
    print(f"{m} mixed steps: mean span {span / m:.1f} us, kernel time {busy / m:.1f} us "
          f"({100 * busy / max(span, 1e-9):.1f}% busy), {sum(len(st) for st in mixed) / m:.0f} kernels")
    print(f"{'kernel (mixed steps)':60s} {'calls/step':>10} {'us/step':>9} {'avg_us':>8}")
    for n, (k, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"{n:60s} {k / m:10.1f} {d / m:9.1f} {d / k:8.2f}")
    print()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=200, help="decode steps averaged (the last N)")
    ap.add_argument("--first", default="embed_rmsnorm", help="kernel that opens a step")
    a = ap.parse_args()
    rows = _load(a.db)
    # split into steps at the step-opening kernel
    steps, cur = [], []
    for name, s, e in rows:
        if a.first in name and cur:
            steps.append(cur)
            cur = []
        cur.append((_short(name), s, e))
    if cur:
        steps.append(cur)
    mixed = [st for st in steps if any("prefill" in n for n, _, _ in st)]
    if mixed:
        _mixed_summary(mixed)
    # decode steps: no prefill kernels, and the most common kernel count
    dec = [st for st in steps if not any("prefill" in n or "packed_gemm" in n for n, _, _ in st)]
    if not dec:
        print("no decode steps found")
        return
    counts = defaultdict(int)
    for st in dec:
        counts[len(st)] += 1
    n_k = max(counts, key=counts.get)
    dec = [st for st in dec if len(st) == n_k][-a.steps:]
    dur = [0.0] * n_k
    gap = [0.0] * n_k
    names = [n for n, _, _ in dec[0]]
    span = 0.0
    for st in dec:
        span += (st[-1][2] - st[0][1]) / 1e3
        for i, (n, s, e) in enumerate(st):
            dur[i] += (e - s) / 1e3
            if i:
                gap[i] += max(0.0, (s - st[i - 1][2]) / 1e3)
    m = len(dec)
    dur = [d / m for d in dur]
    gap = [g / m for g in gap]
    print(f"{m} decode steps of {n_k} kernels: step span {span / m:.1f} us, "
          f"kernel time {sum(dur):.1f} us, gaps {sum(gap):.1f} us")
    # aggregate by kernel name (the layer repeats)
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for n, d, g in zip(names, dur, gap):
        agg[n][0] += 1
        agg[n][1] += d
        agg[n][2] += g
    print(f"{'kernel':60s} {'calls':>5} {'us/step':>9} {'avg_us':>8} {'gap_before_avg':>14}")
    for n, (k, d, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:60s} {k:5d} {d:9.1f} {d / k:8.2f} {g / k:14.2f}")
    # one layer in order (positions of the second layer)
    print("\nlayer 2 in order (mean duration / gap before, us):")
    per_layer = (n_k - 1) // 32 if n_k > 40 else 0
    if per_layer:
        base = 1 + per_layer
        for i in range(base, base + per_layer):
            print(f"  {names[i]:60s} {dur[i]:8.2f} {gap[i]:8.2f}")


if __name__ == "__main__":
    main()
