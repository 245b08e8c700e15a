"""Plain-PyTorch fp32 reference implementations of every native op.

They define the semantics the gfx950 kernels in ``csrc/kernels`` must match
(numerics tests compare the two), and they are the compute path of the CPU
backend (BASELINE config 1: a llama3.2-1b-shaped model streaming over /ws/llm
with no GPU).  All math is done in fp32 and rounded once to the storage dtype,
mirroring the kernels.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    n = (xf * inv).to(x.dtype)
    return (n.float() * w.float()).to(x.dtype)


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    r = (x.float() + residual.float()).to(x.dtype)
    return rmsnorm(r, w, eps), r


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    inter = gu.shape[-1] // 2
    g = gu[..., :inter].float()
    u = gu[..., inter:].float()
    return (g * torch.sigmoid(g) * u).to(gu.dtype)


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None,
                 device=None) -> torch.Tensor:
    """fp32 [max_pos, head_dim] table = [cos | sin] of the rotate_half convention.

    ``scaling`` follows the Llama-3.1 "llama3" rope_scaling dict (factor,
    low_freq_factor, high_freq_factor, original_max_position_embeddings).
    """
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv_freq
        scaled = torch.where(wl > lo_wl, inv_freq / factor, inv_freq)
        smooth = (old / wl - lo) / (hi - lo)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv_freq = torch.where(is_mid, mid, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv_freq)
    return torch.cat([freqs.cos(), freqs.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x: [T, H, D] -> rotated (fp32 math, x.dtype output)."""
    d = x.shape[-1]
    half = d // 2
    cs = cos_sin[positions.long()]  # [T, D]
    cos = cs[:, None, :half]
    sin = cs[:, None, half:]
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


FP8_MAX = 448.0   # float8_e4m3fn's largest finite value


def to_cache(x: torch.Tensor, cache: torch.Tensor) -> torch.Tensor:
    """x in the cache's dtype; fp8 caches clamp to the format's range first (a plain
    cast turns an out-of-range value into NaN, as gfx950's converter does)."""
    if cache.dtype == torch.float8_e4m3fn:
        return x.float().clamp(-FP8_MAX, FP8_MAX).to(cache.dtype)
    return x.to(cache.dtype)


def rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, nq, nkv, head_dim):
    """In place: rotate q inside ``qkv``; write rotated k and v into the paged caches."""
    t = qkv.shape[0]
    if t == 0:
        return
    d = head_dim
    q = qkv[:, : nq * d].view(t, nq, d)
    k = qkv[:, nq * d: (nq + nkv) * d].view(t, nkv, d)
    v = qkv[:, (nq + nkv) * d: (nq + 2 * nkv) * d].view(t, nkv, d)
    q.copy_(apply_rope(q, positions, cos_sin))
    kr = apply_rope(k, positions, cos_sin)
    slots = slot_mapping[:t].long()
    keep = slots >= 0
    if keep.any():
        bs = k_cache.shape[2]
        s = slots[keep]
        blk, off = s // bs, s % bs
        k_cache[blk, :, off, :] = to_cache(kr[keep], k_cache)
        v_cache[blk, :, :, off] = to_cache(v[keep], v_cache)   # V blocks transposed: [blocks, nkv, D, bs]


def _gather_kv(cache, table_row, length, transposed: bool = False):
    """[length, H, D] rows of one sequence; ``transposed``: V blocks [H, D, bs]."""
    if transposed:
        cache = cache.transpose(2, 3)
    bs = cache.shape[2]
    nblk = (length + bs - 1) // bs
    blocks = table_row[:nblk].long()
    kv = cache[blocks]  # [nblk, H, bs, D]
    kv = kv.permute(0, 2, 1, 3).reshape(nblk * bs, cache.shape[1], cache.shape[3])
    return kv[:length]


def paged_attention(q: torch.Tensor, k_cache, v_cache, block_tables, seq_lens, q_start_loc,
                    scale: float) -> torch.Tensor:
    """Causal varlen attention over the paged cache (K blocks [nkv, bs, D], V
    blocks transposed [nkv, D, bs]).

    q: [T, nq, D] (new tokens of every sequence, packed by q_start_loc)
    Each sequence b attends to kv positions [0, seq_lens[b]); its new tokens
    sit at the end (positions seq_len - q_len ...).  Returns [T, nq, D].
    """
    t, nq, d = q.shape
    out = torch.empty_like(q)
    nkv = k_cache.shape[1]
    g = nq // nkv
    qsl = q_start_loc.tolist()
    sl = seq_lens.tolist()
    for b in range(len(sl)):
        q0, q1 = qsl[b], qsl[b + 1]
        if q1 == q0:
            continue
        L = sl[b]
        k = _gather_kv(k_cache, block_tables[b], L).float()  # [L, nkv, D]
        v = _gather_kv(v_cache, block_tables[b], L, transposed=True).float()
        qq = q[q0:q1].float()  # [ql, nq, D]
        ql = q1 - q0
        k = k.repeat_interleave(g, dim=1)
        v = v.repeat_interleave(g, dim=1)
        s = torch.einsum("qhd,khd->hqk", qq, k) * scale
        qpos = torch.arange(L - ql, L, device=q.device)[:, None]
        kpos = torch.arange(L, device=q.device)[None, :]
        s = s.masked_fill((kpos > qpos)[None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        out[q0:q1] = torch.einsum("hqk,khd->qhd", p, v).to(q.dtype)
    return out


def sample(logits: torch.Tensor, temperature, top_p, top_k, seeds, steps,
           mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Reference sampler (CPU backend).  Same contract as the HIP kernel:
    temperature <= 0 -> argmax (lowest id on ties); else top-k, then top-p over
    the survivors, then a draw from the renormalised distribution.  The draw is
    seeded by (seed, step) so it is reproducible, but it does not reproduce the
    kernel's random stream bit for bit (tests compare distributions)."""
    x = logits.float().clone()
    b, v = x.shape
    if mask is not None:
        bits = mask[:b].to(torch.int64) & 0xFFFFFFFF
        ids = torch.arange(v, device=x.device)
        allowed = ((bits[:, ids // 32] >> (ids % 32)) & 1).bool()
        x = x.masked_fill(~allowed, float("-inf"))
    out = torch.empty(b, dtype=torch.int32, device=x.device)
    for i in range(b):
        row = x[i]
        t = float(temperature[i])
        if t <= 0:
            out[i] = int(torch.argmax(row))
            continue
        z = (row - row.max()) / t
        k = int(top_k[i])
        keep = torch.isfinite(z)
        if 0 < k < v:
            kth = torch.topk(row, k).values[-1]
            keep &= row >= kth
        p = float(top_p[i])
        if p < 1.0:
            pr = torch.softmax(z.masked_fill(~keep, float("-inf")), dim=-1)
            sp, si = torch.sort(pr, descending=True)
            cum = torch.cumsum(sp, 0)
            n_keep = int(torch.searchsorted(cum, torch.tensor(p, dtype=cum.dtype)).item()) + 1
            thr = sp[min(n_keep, v) - 1]
            keep &= pr >= thr
        probs = torch.softmax(z.masked_fill(~keep, float("-inf")), dim=-1)
        gen = torch.Generator(device="cpu")
        gen.manual_seed((int(seeds[i]) * 1000003 + int(steps[i])) & 0x7FFFFFFFFFFFFFFF)
        out[i] = int(torch.multinomial(probs.cpu(), 1, generator=gen).item())
    return out
