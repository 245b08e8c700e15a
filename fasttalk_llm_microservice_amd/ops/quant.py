"""W4A16 weight quantization (E9 / K14): AWQ-format int4, group 128, with zero points.

Replaces vLLM's ``--quantization awq`` (``docker-compose.vllm.yml:45-46``), which the
reference's default model needs (``hugging-quants/Meta-Llama-3.1-8B-Instruct-AWQ-INT4``,
``app/utils/config.py:93-96``).

* :func:`quantize_w4`: round-to-nearest asymmetric int4 per (row, 128-group), for
  random-init weights (and any bf16 checkpoint, ``ENGINE_QUANTIZATION=w4``).
* :func:`awq_unpack` / :func:`awq_pack`: the AutoAWQ "GEMM" checkpoint layout
  (``qweight`` [K, N/8] int32, ``qzeros`` [K/G, N/8] int32, ``scales`` [K/G, N] fp16,
  nibble i of a packed word = column 8c + (0, 2, 4, 6, 1, 3, 5, 7)[i]).  No AWQ
  checkpoint is available offline, so parity with a real one is unpinned; the
  round trip is tested against :func:`awq_pack`.
* :func:`pack_w4`: (q, z, s) -> the MFMA-fragment image ``w4a16.hip`` streams.
* :class:`W4Weight` holds one packed projection; :func:`w4_gemm` / :func:`w4_dequant`
  dispatch to the HIP kernels, or to a dequantize + matmul reference on the CPU.
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Tuple

import torch

GROUP = 128
AWQ_ORDER = (0, 2, 4, 6, 1, 3, 5, 7)   # nibble i of an AWQ word holds column AWQ_ORDER[i]
_NIBBLE_K = (0, 2, 4, 6, 1, 3, 5, 7)   # nibble p of one of our words holds k offset _NIBBLE_K[p]


@dataclasses.dataclass
class W4Weight:
    wq: torch.Tensor   # int32 [N/16 * K/128 * 64 * 4]  packed nibbles
    sz: torch.Tensor   # fp32 [N/16, K/128, 16, 2]      (scale, 128 + zero)
    n: int
    k: int

    @property
    def shape(self) -> Tuple[int, int]:
        return (self.n, self.k)

    def nbytes(self) -> int:
        return self.wq.numel() * 4 + self.sz.numel() * 4


def quantize_w4(w: torch.Tensor, group: int = GROUP):
    """[N, K] float -> (q uint8 [N, K], z uint8 [N, K/g], s fp32 [N, K/g]) with
    w ~= (q - z) * s (round to nearest, asymmetric per row and group)."""
    n, k = w.shape
    assert k % group == 0
    # fp64: correctly rounded on every backend, so a GPU and a CPU quantization of
    # the same weights agree bit for bit
    wf = w.double().view(n, k // group, group)
    mn = wf.amin(-1).clamp(max=0.0)
    mx = wf.amax(-1).clamp(min=0.0)
    s = ((mx - mn) / 15.0).clamp(min=1e-8).float().double()
    z = torch.round(-mn / s).clamp(0, 15)
    q = (torch.round(wf / s.unsqueeze(-1)) + z.unsqueeze(-1)).clamp(0, 15)
    return q.view(n, k).to(torch.uint8), z.to(torch.uint8), s.float()


def dequantize_w4(q: torch.Tensor, z: torch.Tensor, s: torch.Tensor, group: int = GROUP):
    n, k = q.shape
    w = (q.float().view(n, k // group, group) - z.float().unsqueeze(-1)) * s.float().unsqueeze(-1)
    return w.view(n, k)


def _to_i32(v: torch.Tensor) -> torch.Tensor:
    """int64 holding uint32 bit patterns -> int32 with the same bits."""
    return torch.where(v >= 2 ** 31, v - 2 ** 32, v).to(torch.int32)


def _nibbles(words: torch.Tensor) -> torch.Tensor:
    """int32 [...] -> int64 [..., 8] nibbles (nibble i = bits 4i..4i+3)."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    shifts = torch.arange(0, 32, 4, device=words.device)
    return (w.unsqueeze(-1) >> shifts) & 15


def _pack_nibbles(nib: torch.Tensor) -> torch.Tensor:
    """int [..., 8] (values 0..15, nibble i at bits 4i) -> int32 [...]."""
    shifts = torch.arange(0, 32, 4, device=nib.device)
    return _to_i32((nib.to(torch.int64) << shifts).sum(-1))


def pack_w4(q: torch.Tensor, z: torch.Tensor, s: torch.Tensor) -> W4Weight:
    """(q, z, s) -> the kernel image.  wq[tile][grp][lane][word], lane = g*16 + r,
    word = 2*step + half, nibble p = k offset 128 grp + 64 step + 16 g + 8 half +
    _NIBBLE_K[p] of column 16 tile + r."""
    n, k = q.shape
    assert n % 16 == 0 and k % GROUP == 0, "W4 needs N % 16 == 0 and K % 128 == 0"
    dev = q.device
    # (tile, r, grp, step, g, half, e) -> (tile, grp, g, r, step, half, e)
    t = q.to(torch.int64).view(n // 16, 16, k // 128, 2, 4, 2, 8).permute(0, 2, 4, 1, 3, 5, 6)
    t = t[..., list(_NIBBLE_K)]
    wq = _pack_nibbles(t).contiguous().view(-1)
    sz = torch.stack([s.float(), z.float() + 128.0], -1)          # [N, G, 2]
    sz = sz.view(n // 16, 16, k // 128, 2).permute(0, 2, 1, 3).contiguous()
    return W4Weight(wq.to(dev), sz.to(dev), n, k)


def unpack_w4(w: W4Weight):
    """Inverse of :func:`pack_w4` (tests, checkpoint export)."""
    n, k = w.n, w.k
    nib = _nibbles(w.wq.view(n // 16, k // 128, 4, 16, 2, 2))      # (tile, grp, g, r, step, half, p)
    inv = [0] * 8
    for p, off in enumerate(_NIBBLE_K):
        inv[off] = p
    nib = nib[..., inv]                                             # e order
    q = nib.permute(0, 3, 1, 4, 2, 5, 6).contiguous().view(n, k).to(torch.uint8)
    sz = w.sz.view(n // 16, k // 128, 16, 2).permute(0, 2, 1, 3).reshape(n, k // 128, 2)
    return q, (sz[..., 1] - 128.0).round().to(torch.uint8), sz[..., 0].contiguous()


# ------------------------------------------------------------------ AutoAWQ layout
def awq_unpack(qweight: torch.Tensor, qzeros: torch.Tensor, scales: torch.Tensor):
    """AutoAWQ GEMM tensors of one linear (in K, out N) -> (q [N, K], z [N, G], s [N, G])."""
    kk, n8 = qweight.shape
    inv = [0] * 8
    for i, col in enumerate(AWQ_ORDER):
        inv[col] = i
    q = _nibbles(qweight)[..., inv].reshape(kk, n8 * 8)            # [K, N]
    z = _nibbles(qzeros)[..., inv].reshape(qzeros.shape[0], n8 * 8)  # [G, N]
    return (q.t().contiguous().to(torch.uint8), z.t().contiguous().to(torch.uint8),
            scales.float().t().contiguous())


def awq_pack(q: torch.Tensor, z: torch.Tensor, s: torch.Tensor):
    """(q [N, K], z [N, G], s [N, G]) -> AutoAWQ (qweight, qzeros, scales fp16)."""
    n, k = q.shape
    qk = q.t().to(torch.int64).reshape(k, n // 8, 8)[..., list(AWQ_ORDER)]
    zg = z.t().to(torch.int64).reshape(z.shape[1], n // 8, 8)[..., list(AWQ_ORDER)]
    return _pack_nibbles(qk), _pack_nibbles(zg), s.t().contiguous().to(torch.float16)


# ------------------------------------------------------------------ compute
def w4_dequant(w: W4Weight, out: Optional[torch.Tensor] = None,
               dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    if w.wq.is_cuda:
        from . import native

        if out is None:
            out = torch.empty(w.n, w.k, dtype=torch.bfloat16, device=w.wq.device)
        native().w4_dequant(w.wq, w.sz, out)
        return out
    q, z, s = unpack_w4(w)
    r = dequantize_w4(q, z, s).to(dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


def w4_gemm(x: torch.Tensor, w: W4Weight, out=None, ws=None, splits: int = 1, nt: int = 1,
            xr: int = 0, silu: bool = False):
    """y = x dequant(w)^T for M <= 64 rows.  With ``ws`` the kernel leaves fp32
    slabs ([splits, M, N]) for a fused epilogue; otherwise returns bf16 ``out``.
    ``xr`` picks the kernel (w4a16.hip): 0 the register kernel, 1 "xr" (x chunks in
    LDS, 17..64 rows), 4 / 5 "mh" (two tiles per wave, rows over wave pairs; weight
    ring 2 with two x chunks in flight / ring 3).  ``silu``: the LDS kernels' SiLU
    epilogue on a gate/up image interleaved in 16-row groups (h = silu(gate) * up)."""
    if not x.is_cuda:
        y = x @ w4_dequant(w, dtype=x.dtype).t()
        if silu:
            g, u = y.view(y.shape[0], -1, 2, 16).unbind(2)
            y = (torch.nn.functional.silu(g.float()) * u.float()).to(x.dtype).reshape(y.shape[0], -1)
        return y
    from . import native

    if ws is None and out is None:
        out = torch.empty(x.shape[0], w.n // 2 if silu else w.n, dtype=x.dtype, device=x.device)
    native().w4_gemm(x, w.wq, w.sz, w.n, out, ws, splits, nt, int(xr), silu)
    return out if ws is None else ws
