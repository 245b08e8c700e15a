"""Summarises an engine step trace (FT_STEP_TRACE=<path> json written at shutdown):
time in pipelined decode steps, synchronous decode / mixed (prefill) steps, and
host time between steps, over the last --last-s seconds of the trace.

python bench/step_trace_summary.py gpurun_out/trace.json --last-s 15
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last-s", type=float, default=15.0)
    a = ap.parse_args()
    tr = json.load(open(a.path))
    if not tr:
        print("empty trace")
        return
    arrivals = [r for r in tr if r[0] == "arrive"]
    tr = [r for r in tr if len(r) == 6]
    end = tr[-1][2]
    tr = [r for r in tr if r[1] >= end - a.last_s]
    arrivals = [r for r in arrivals if r[1] >= tr[0][1]]
    wall = tr[-1][2] - tr[0][1]
    kinds = {}
    between = 0.0
    for i, (kind, t0, t1, nd, ptok, npre) in enumerate(tr):
        k = kinds.setdefault(kind, {"n": 0, "s": 0.0, "rows": 0, "ptok": 0, "npre": 0})
        k["n"] += 1
        k["s"] += t1 - t0
        k["rows"] += nd
        k["ptok"] += ptok
        k["npre"] += npre
        if i:
            between += max(0.0, t0 - tr[i - 1][2])
    print(f"window {wall:.2f} s, {len(tr)} steps, between steps {1e3 * between:.1f} ms "
          f"({100 * between / wall:.1f}%)")
    for kind, k in sorted(kinds.items()):
        print(f"  {kind:9s} n {k['n']:6d}  total {k['s']:7.2f} s ({100 * k['s'] / wall:5.1f}%)  "
              f"avg {1e3 * k['s'] / k['n']:7.2f} ms  decode rows {k['rows'] / k['n']:6.1f}  "
              f"prefill tok {k['ptok'] / k['n']:7.1f}  prefill seqs {k['npre'] / k['n']:5.1f}")
    # pipeline restarts: a decode_p step whose predecessor was not decode_p
    starts = sum(1 for i in range(1, len(tr)) if tr[i][0] == "decode_p" and tr[i - 1][0] != "decode_p")
    print(f"  pipeline (re)starts {starts}, request arrivals {len(arrivals)}")
    # mixed / prefill steps by total GEMM rows (decode rows + prefill tokens): the
    # prefill GEMMs tile M by 256, so steps just past a multiple of 256 pay a tile row
    hist = {}
    for kind, t0, t1, nd, ptok, npre in tr:
        if ptok:
            h = hist.setdefault(min(2048, (nd + ptok + 255) // 256 * 256), [0, 0.0, 0])
            h[0] += 1
            h[1] += t1 - t0
            h[2] += nd + ptok
    for lim in sorted(hist):
        n, s, rows = hist[lim]
        print(f"  rows <= {lim:5d}{'+' if lim == 2048 else ' '} n {n:5d}  avg {1e3 * s / n:7.2f} ms  "
              f"avg rows {rows / n:7.1f}  total {s:6.2f} s")


if __name__ == "__main__":
    main()
