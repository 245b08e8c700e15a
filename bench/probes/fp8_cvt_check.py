"""Compares bench/probes/fp8_cvt_probe's output (gfx950 fp8 conversions) with
torch.float8_e4m3fn: decode of all 256 codes at scales 1 / 0.5 / 3 (bf16 result),
and encode of a float ramp over [-500, 500] (round-to-nearest-even, saturation)."""
import sys

import torch

lines = open(sys.argv[1]).read().split("\n")
codes = torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).float()
for ln in lines:
    if ln.startswith("dec"):
        parts = ln.split()
        s = float(parts[1])
        got = torch.tensor([int(v) for v in parts[2:]], dtype=torch.int32).to(torch.int16).view(torch.bfloat16).float()
        want = (codes * s).bfloat16().float()
        fin = torch.isfinite(want)
        bad = ((got != want) & fin).sum().item()
        print(f"decode scale {s}: {bad} mismatches on {fin.sum().item()} finite codes; NaN codes -> "
              f"{got[~fin].tolist()}")
    if ln.startswith("enc"):
        got = torch.tensor([int(v) for v in ln.split()[1:]], dtype=torch.uint8)
        x = -500 + 0.5 * torch.arange(got.numel(), dtype=torch.float32)
        want = x.to(torch.float8_e4m3fn).view(torch.uint8)
        inr = x.abs() <= 448
        bad = (got != want) & inr
        print(f"encode: {bad.sum().item()} mismatches in range; out of range -> "
              f"{sorted(set(got[~inr].view(torch.float8_e4m3fn).float().tolist()))[:6]}")
        if bad.any():
            i = bad.nonzero()[:5, 0]
            print(" e.g.", x[i].tolist(), got[i].view(torch.float8_e4m3fn).float().tolist(),
                  want[i].view(torch.float8_e4m3fn).float().tolist())
