"""Print value / p50 / p99 / decode step of bench.py JSON lines in gpurun_out logs.
python bench/bsum.py gpurun_out/a.log gpurun_out/b.log"""
import json
import sys

for p in sys.argv[1:]:
    try:
        lines = [l for l in open(p).read().splitlines() if l.startswith("{")]
        d = json.loads(lines[-1])
        tool = d.get("tool_turns")
        extra = f"  tool p50 {tool['p50_ttft_ms']:6.1f} p99 {tool['p99_ttft_ms']:6.1f}" if tool else ""
        print(f"{p:32s} {d['value']:9.1f} tok/s  p50 {d['p50_ttft_ms']:7.1f}  p99 {d['p99_ttft_ms']:7.1f}  "
              f"step {d['engine_decode_step_ms']:6.2f}  engine_ttft {d.get('p50_engine_ttft_ms')}{extra}")
    except Exception as e:  # noqa
        print(p, "->", e)
