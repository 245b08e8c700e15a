"""Op dispatch: GPU tensors -> gfx950 HIP kernels (``_C``), CPU tensors -> the
fp32 PyTorch references in :mod:`.reference`.

There is deliberately no silent fallback for GPU tensors: if the native
extension is missing or fails to load on a GPU host the first op raises, so a
run can never pass on an eager PyTorch path while claiming the HIP kernels.
"""
from __future__ import annotations

import os
import threading
from typing import Optional

import numpy as np
import torch

from . import reference as ref

_lock = threading.Lock()
_C = None
_C_err: Optional[BaseException] = None


def kernel_checks_requested() -> bool:
    """``FT_KERNEL_CHECKS=1``: load the bounds-checked kernel build ``_C_checked``
    (csrc/include/ft_common.h; the runner reads its error word after every step)."""
    return os.environ.get("FT_KERNEL_CHECKS", "0").strip().lower() in ("1", "true", "yes", "on")


def native():
    """Return the loaded ``_C`` extension (``_C_checked`` under FT_KERNEL_CHECKS=1),
    building it in-tree if allowed."""
    global _C, _C_err
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        checked = kernel_checks_requested()
        name = "_C_checked" if checked else "_C"
        import importlib

        try:
            mod = importlib.import_module(f"..{name}", __package__)
        except ImportError as e:  # pragma: no cover - depends on build state
            if os.environ.get("FT_AUTOBUILD", "1") != "0":
                from .build import build_kernels

                build_kernels(verbose=True, checked=checked)
                mod = importlib.import_module(f"..{name}", __package__)
            else:
                _C_err = e
                raise RuntimeError(
                    f"fasttalk native extension {name} is not built; run "
                    "`python -m fasttalk_llm_microservice_amd.ops.build`") from e
        _C = mod
        return _C


def native_available() -> bool:
    try:
        native()
        return True
    except Exception:
        return False


# ---------------------------------------------------------------------------------
# norms / activations
# ---------------------------------------------------------------------------------

def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None):
    if x.is_cuda:
        if out is None:
            out = torch.empty_like(x)
        if x.shape[1] % 2048 == 0:
            native().row_rmsnorm(out, x, None, 1, None, w, x.shape[0], eps)
        else:
            native().rmsnorm(out, x, w, eps)
        return out
    r = ref.rmsnorm(x, w, eps)
    if out is not None:
        out.copy_(r)
        return out
    return r


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """residual <- x + residual;  x <- rmsnorm(residual) * w   (both in place)."""
    if x.is_cuda:
        if x.shape[1] % 2048 == 0:
            native().row_rmsnorm(x, x, None, 1, residual, w, x.shape[0], eps)
        else:
            native().fused_add_rmsnorm(x, x, residual, w, eps)
        return x, residual
    y, r = ref.fused_add_rmsnorm(x, residual, w, eps)
    residual.copy_(r)
    x.copy_(y)
    return x, residual


def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None, interleaved: bool = False):
    """silu(gate) * up of [M, 2I] gate_up rows: halves [gate | up], or ``interleaved``
    groups of 16 (interleave_gate_up(w, 1), the packed model's gate_up image)."""
    if gu.is_cuda:
        if out is None:
            out = torch.empty(gu.shape[0], gu.shape[1] // 2, dtype=gu.dtype, device=gu.device)
        native().silu_mul(out, gu, interleaved)
        return out
    if interleaved:
        m, two_i = gu.shape
        v = gu.reshape(m, two_i // 32, 2, 16)
        gu = torch.cat([v[:, :, 0].reshape(m, -1), v[:, :, 1].reshape(m, -1)], dim=1)
    r = ref.silu_mul(gu)
    if out is not None:
        out.copy_(r)
        return out
    return r


# ---------------------------------------------------------------------------------
# rotary + paged KV
# ---------------------------------------------------------------------------------

def rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, nq, nkv, head_dim):
    if qkv.is_cuda:
        native().rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, nq, nkv,
                               head_dim)
    else:
        ref.rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, nq, nkv,
                          head_dim)


# Batch-invariant decode attention: every (sequence, kv head) is cut into pieces of
# this many 16-token tiles from its first token (csrc/kernels/attn_decode.hip piece
# mode), whatever the rest of the batch.
DECODE_INV_PIECE = 32


def decode_workspace(batch: int, nq: int, nkv: int, head_dim: int, waves: Optional[int] = None,
                     piece: int = 0, max_len: int = 0):
    """(tmp_out, tmp_ml) element counts of the decode kernel's partial workspace:
    one fp32 slot per (sequence, kv head) plus one per wave of the grid
    (csrc/kernels/attn_decode.hip), each holding the G = nq / nkv heads.  With
    ``piece`` (batch-invariant mode) one slot per piece of a ``max_len`` sequence."""
    if waves is None:
        waves = native().decode_waves() if native_available() else 0
    slots = batch * nkv + waves
    if piece > 0:
        tiles = -(-max_len // 16)
        slots = max(slots, batch * nkv * -(-tiles // piece))
    g = nq // nkv
    return slots * g * head_dim, slots * g * 2


def prefill_tile_tokens(nq: int, nkv: int) -> int:
    """Query tokens per prefill workgroup (256 MFMA rows of token x GQA head)."""
    return 256 // (nq // nkv)


def decode_counters(batch: int, nkv: int, device) -> torch.Tensor:
    """Zeroed int32 tickets of the decode kernel's in-launch combine (one per
    sequence x kv head; the kernel leaves them zeroed)."""
    return torch.zeros(max(1, batch * nkv), dtype=torch.int32, device=device)


def decode_attention(out, q, k_cache, v_cache, block_tables, seq_lens, tmp_out, tmp_ml, nq, nkv,
                     head_dim, scale, counters: Optional[torch.Tensor] = None, piece: int = 0):
    """out[b] = attention of the single new query of sequence b (q: [B, >=nq*D] rows).
    k_cache [blocks, nkv, bs, D]; v_cache [blocks, nkv, D, bs] (transposed blocks).
    ``counters`` (decode_counters): merge shared segments inside the launch instead
    of a second combine kernel.  ``piece`` > 0: batch-invariant partition (fixed
    pieces of that many tiles per sequence; needs counters and a workspace from
    decode_workspace(piece=...))."""
    if q.is_cuda:
        native().paged_decode_attention(out, q, k_cache, v_cache, block_tables, seq_lens, tmp_out,
                                        tmp_ml, nq, nkv, head_dim, scale, counters, piece)
        return out
    b = q.shape[0]
    qq = q[:, : nq * head_dim].reshape(b, nq, head_dim)
    qsl = torch.arange(b + 1, dtype=torch.int32)
    o = ref.paged_attention(qq, k_cache, v_cache, block_tables, seq_lens[:b], qsl, scale)
    out[:b, : nq * head_dim].copy_(o.reshape(b, nq * head_dim))
    return out


def prefill_attention(out, q, k_cache, v_cache, block_tables, seq_lens, q_start_loc, tile_info,
                      num_tiles, nq, nkv, head_dim, scale, part_o=None, part_ml=None, combine=None,
                      num_combine: int = 0, num_partials: int = 0, invariant: bool = False):
    """Varlen causal attention of the new tokens over their paged history.
    ``tile_info``: the work items of build_prefill_tiles (4 int32 each); split-KV
    items leave fp32 partials in ``part_o`` / ``part_ml`` (prefill_partials) that
    the ``combine`` list merges (csrc/kernels/attn_prefill.hip).  ``invariant``:
    per-row rescale decisions (batch-invariant mode, with a fixed_chunk plan)."""
    if q.is_cuda:
        native().prefill_attention(out, q, k_cache, v_cache, block_tables, seq_lens, q_start_loc,
                                   tile_info, num_tiles, nq, nkv, head_dim, scale, part_o, part_ml,
                                   combine, num_combine, num_partials, invariant)
        return out
    t = q.shape[0]
    qq = q[:, : nq * head_dim].reshape(t, nq, head_dim)
    o = ref.paged_attention(qq, k_cache, v_cache, block_tables, seq_lens, q_start_loc, scale)
    out[:t, : nq * head_dim].copy_(o.reshape(t, nq * head_dim))
    return out


PREFILL_BK = 64          # KV tokens per tile of the prefill kernel
PREFILL_ROWS = 256       # MFMA rows (query token x GQA head) per work item
PREFILL_MAX_PARTIALS = 128


def prefill_partials(nkv: int, head_dim: int, max_partials: int = PREFILL_MAX_PARTIALS):
    """(part_o, part_ml) fp32 element counts of the split-KV workspace."""
    return max_partials * nkv * PREFILL_ROWS * head_dim, max_partials * nkv * PREFILL_ROWS * 2


# per-work-item overhead of the prefill kernel in 64-token KV tiles (Q load, DMA ramp,
# partial store + its combine), for the round-aware split plan below.  Swept on MI355X
# (profiles/prefill_item_tiles_r04.log): 2 = 1 at every chat-turn shape but one, where it
# plans one round instead of two (4 x 150 new over 1.5k: 46.9 vs 58.9 us)
PREFILL_ITEM_TILES = float(os.environ.get("FT_PREFILL_ITEM_TILES", "2.0"))
PREFILL_MAX_ROUNDS = 4
PREFILL_ROUND_BLIND = os.environ.get("FT_PREFILL_ROUND_BLIND", "0") == "1"


# Batch-invariant prefill plan: KV ranges cut at absolute multiples of this many
# 64-token tiles (1024 tokens), so a query row sees the same pieces in the same
# order whatever chunk, query block or batch it is computed in.
PREFILL_INV_CHUNK = 16


def build_prefill_tiles(q_lens, tile_tokens: int, seq_lens=None, nkv: int = 8, num_cus: int = 256,
                        max_partials: int = PREFILL_MAX_PARTIALS, min_split_tiles: int = 4,
                        fixed_chunk: int = 0):
    """Host plan of the prefill kernel grid: (items, combine).

    ``fixed_chunk`` (batch-invariant mode): every block's KV range is cut at
    absolute multiples of that many tiles (pieces past a row's position are masked
    no-ops in the merge) and the plan never falls back to an unsplit item; raises
    if the partial slots run out.

    items: [(seq, first query token, kv_lo_tile << 16 | kv_hi_tile, partial slot)],
    one per (query block, KV range); combine: [(seq, first query token, first slot,
    splits)] for query blocks whose KV range is split over several workgroups.
    Without ``seq_lens`` no range is split.  A chat turn prefills ~100 tokens over
    thousands of cached ones: ~2 query blocks per prompt, so a 10-prompt step would
    be 160 workgroups each streaming a whole history alone -- the ranges are cut.

    The kernel runs ONE workgroup per CU (``attn_prefill.hip``: 8 waves, 144 KiB of
    LDS), so the grid executes in rounds of ``num_cus`` workgroups (= num_cus / nkv
    items): for 1..PREFILL_MAX_ROUNDS rounds the smallest chunk (>= min_split_tiles
    tiles) whose items fit is found and the plan with the least estimated makespan
    (rounds x (longest item + PREFILL_ITEM_TILES)) wins.  The earlier plan aimed at
    ~2 workgroups per CU and rounded every block's split up, e.g. 520 workgroups for
    5 prompts x 107 tokens over 3k: a third round for 8 workgroups."""
    blocks = []
    for b, ql in enumerate(q_lens):
        ql = int(ql)
        for s in range(0, ql, tile_tokens):
            if seq_lens is None:
                nkt = 0
            else:
                L = int(seq_lens[b])
                kv_end = min(L, L - ql + s + min(tile_tokens, ql - s))
                nkt = (kv_end + PREFILL_BK - 1) // PREFILL_BK
            blocks.append((b, s, nkt))
    items, combine = [], []
    if fixed_chunk > 0:
        slots = 0
        for b, s, nkt in blocks:
            ns = -(-nkt // fixed_chunk)
            if ns <= 1 or seq_lens is None:
                items.append((b, s, 0xFFFF, -1))
                continue
            if slots + ns > max_partials:
                raise RuntimeError(f"batch-invariant prefill plan needs more than {max_partials} "
                                   "partial slots (fewer batched tokens per step)")
            combine.append((b, s, slots, ns))
            for j in range(ns):
                items.append((b, s, ((j * fixed_chunk) << 16) | min((j + 1) * fixed_chunk, nkt),
                              slots + j))
            slots += ns
        return items, combine
    per_round = max(1, num_cus // max(1, nkv))
    chunk = 0
    nk_lo = min(n for _, _, n in blocks) if blocks else 0
    nk_hi = max(n for _, _, n in blocks) if blocks else 0
    # the round model assumes near-equal items: a causal prompt's early blocks (a few
    # tiles each) make the greedy dispatch far from it (1 x 2048 fresh tokens ran 103
    # vs 91 us on the round-aware plan), so ranges that differ by more than 2x keep
    # the round-blind split (profiles/prefill_round_plan_r03.log)
    blind = PREFILL_ROUND_BLIND or nk_lo * 2 < nk_hi
    if seq_lens is not None and blocks and blind:
        # the round-2 plan (~2 workgroups per CU, per-block round-up), for A/B runs
        target = 2 * per_round
        total = sum(n for _, _, n in blocks)
        if len(blocks) < target and total > 0:
            chunk = max(min_split_tiles, -(-total // target))
    elif seq_lens is not None and blocks:   # history-dominated: round-aware split
        nk = np.fromiter((n for _, _, n in blocks), dtype=np.int64, count=len(blocks))
        top = int(nk.max())
        if top > min_split_tiles:
            # candidate chunks: the longest block cut into 1..32 equal parts
            c = np.unique(np.maximum(-(-top // np.arange(1, 33)), min_split_tiles))
            ns = np.maximum(-(-nk[None, :] // c[:, None]), 1)
            n_items = ns.sum(1)
            n_part = np.where(ns > 1, ns, 0).sum(1)
            rounds = -(-n_items // per_round)
            cost = rounds * (c + PREFILL_ITEM_TILES)
            ok = (rounds <= PREFILL_MAX_ROUNDS) & (n_part <= max_partials)
            if ok.any():
                best = int(c[ok][np.argmin(cost[ok])])
                chunk = best if best < top else 0
    slots = 0
    for b, s, nkt in blocks:
        ns = -(-nkt // chunk) if chunk else 1
        if ns > 1 and slots + ns <= max_partials:
            combine.append((b, s, slots, ns))
            for j in range(ns):
                lo, hi = j * nkt // ns, (j + 1) * nkt // ns
                items.append((b, s, (lo << 16) | hi, slots + j))
            slots += ns
        else:
            items.append((b, s, 0xFFFF, -1))
    return items, combine


# ---------------------------------------------------------------------------------
# sampling
# ---------------------------------------------------------------------------------

def sample(logits, temperature, top_p, top_k, seeds, steps, out=None, mask=None):
    if logits.is_cuda:
        b = logits.shape[0]
        if out is None:
            out = torch.empty(b, dtype=torch.int32, device=logits.device)
        native().sample(out, logits, temperature, top_p, top_k, seeds, steps, mask)
        return out
    r = ref.sample(logits, temperature, top_p, top_k, seeds, steps, mask)
    if out is not None:
        out[: r.shape[0]].copy_(r)
        return out
    return r


def kv_block_copy(k_cache, v_cache, pairs: torch.Tensor):
    if k_cache.is_cuda:
        native().kv_block_copy(k_cache, v_cache, pairs)
    else:
        p = pairs.view(-1, 2).long()
        k_cache[p[:, 1]] = k_cache[p[:, 0]]
        v_cache[p[:, 1]] = v_cache[p[:, 0]]


def kv_swap(caches, ptrs, ids: torch.Tensor, staging: torch.Tensor, to_staging: bool):
    """Gathers (``to_staging``) or scatters KV blocks ``ids`` of every layer cache
    to/from ``staging`` [n, 2L, block_elems] (layer-major k0, v0, k1, v1, ...).
    ``caches``: the model's [(k, v)] list; ``ptrs``: their base pointers as an
    int64 tensor on the device (GPU path) or None."""
    n = ids.numel()
    if n == 0:
        return
    flat = [c for kv in caches for c in kv]
    if staging.dtype != flat[0].dtype:   # the kernel sizes a block by the staging dtype
        raise ValueError(f"kv_swap: staging {staging.dtype} vs caches {flat[0].dtype}")
    if staging.is_cuda:
        nblk = flat[0].shape[0]
        native().kv_swap(ptrs, ids, staging, flat[0].numel() // nblk, to_staging, nblk)
        return
    st = staging.view(n, len(flat), -1)
    idx = ids.long()
    for c, cache in enumerate(flat):
        rows = cache.view(cache.shape[0], -1)
        if to_staging:
            st[:, c] = rows[idx]
        else:
            rows[idx] = st[:, c]


# ---------------------------------------------------------------------------------
# decode-shape (M <= 64) weight-streaming GEMM + fused row epilogues
# ---------------------------------------------------------------------------------

# (nt, u) instantiated: u == -3 the "pk" kernel, u == -4 the "xc" kernel, both on
# pre-packed weights (pass pack_weight(w) as w)
SKINNY_CONFIGS = [(1, -3), (2, -3), (4, -3), (1, -4), (2, -4)]
PACKED_VARIANTS = (-3, -4)


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> the MFMA-fragment image the "pk" kernel streams: every 16-column
    x 64-k fragment contiguous, lanes in load order ([N/16][K/64][2][64][8]).
    Returned as an [N, K]-shaped tensor (same bytes, different order)."""
    n, k = w.shape
    assert n % 16 == 0 and k % 64 == 0
    # (t, r, s, g, h, e) -> (t, s, h, g, r, e); lane = g * 16 + r
    p = w.reshape(n // 16, 16, k // 64, 4, 2, 8).permute(0, 2, 4, 3, 1, 5).contiguous()
    return p.view(n, k)


def skinny_gemm(x, w, out=None, ws=None, splits: int = 1, nt: int = 1, u: int = -3):
    """y = x w^T (M <= 64) on a pack_weight() image.  splits > 1 leaves fp32 partial
    slabs in ``ws`` ([splits, M, N]) for a fused epilogue; otherwise writes bf16
    ``out``.  u = -3: "pk" kernel, -4: "xc", -5: "xr" (chunk-pipelined xc),
    -6: "xr" with the SiLU epilogue on an interleave_gate_up(w, 1) image (out is
    h = silu(gate) * up, [M, N / 2]); -7 / -8: -5 / -6 on 8-wave workgroups."""
    if splits == 1 and out is None:
        cols = w.shape[0] // 2 if u in (-6, -8) else w.shape[0]
        out = torch.empty(x.shape[0], cols, dtype=x.dtype, device=x.device)
    native().skinny_gemm(x, w, out, ws, splits, nt, u)
    return out if splits == 1 else ws


def skinny_gemm_xr(x, w, out=None, ws=None, splits: int = 1, nt: int = 2, epi: str = "store",
                   nw: int = 4):
    """The "xr" decode GEMM (M <= 64): epi "store": bf16 out (one split) or fp32 slabs
    [splits, M, N] in ``ws``; "silu": h = silu(gate) * up of an interleave_gate_up(w, 1)
    image, [M, N / 2]."""
    code = {"store": 0, "silu": 1}[epi]
    if out is None and (code == 1 or splits == 1):
        cols = w.shape[0] // 2 if code == 1 else w.shape[0]
        out = torch.empty(x.shape[0], cols, dtype=x.dtype, device=x.device)
    native().skinny_gemm_xr(x, w, out, ws, splits, nt, code, nw)
    return out if code == 1 or splits == 1 else ws


def packed_gemm(x, w, out=None, ws=None, splits: int = 1, epi: str = "store", cfg: int = 0):
    """y = x w^T for any M on a pack_weight() image (csrc/kernels/packed_gemm.hip).
    epi "store": bf16 [M, N]; "slab": fp32 slabs [splits, M, N] in ``ws``; "silu":
    silu(gate) * up of an interleave_gate_up(w, 1) image -> [M, N / 2]."""
    code = {"store": 0, "slab": 1, "silu": 2}[epi]
    if code != 1 and out is None:
        cols = w.shape[0] // 2 if code == 2 else w.shape[0]
        out = torch.empty(x.shape[0], cols, dtype=x.dtype, device=x.device)
    native().packed_gemm(x, w, out, ws, splits, code, cfg)
    return ws if code == 1 else out


def embed_rmsnorm(ids: torch.Tensor, table: torch.Tensor, w: torch.Tensor, eps: float):
    """(rmsnorm(table[ids]) * w, table[ids]): the embedding gather fused with the
    first layer's input norm; the second tensor starts the residual stream."""
    if ids.is_cuda:
        n, h = ids.numel(), table.shape[1]
        out = torch.empty(n, h, dtype=table.dtype, device=table.device)
        res = torch.empty(n, h, dtype=table.dtype, device=table.device)
        native().embed_rmsnorm(out, res, ids, table, w, eps)
        return out, res
    res = torch.nn.functional.embedding(ids.long(), table)
    return ref.rmsnorm(res, w, eps), res


def row_rmsnorm(out, w, eps, rows, x=None, ws=None, splits=1, residual=None):
    native().row_rmsnorm(out, x, ws, splits, residual, w, rows, eps)
    return out


def slab_silu(ws, splits, rows, inter, out, interleaved: bool = False):
    native().slab_silu(ws, splits, rows, inter, out, interleaved)
    return out


def slab_store(ws, splits, rows, cols, out):
    native().slab_store(ws, splits, rows, cols, out)
    return out


def slab_rope_kv(ws, splits, rows, cols, q_out, positions, cos_sin, slot_mapping, k_cache,
                 v_cache, nq, nkv, head_dim, residual=None, eps: float = 0.0):
    """Reduces the QKV split-K slabs, applies RoPE, writes q and the paged K/V.  With
    ``residual`` (fused decode layer) the slabs are scaled by the RMS of the residual
    row first (the input-norm weight is folded into the packed QKV weight)."""
    native().slab_rope_kv(ws, splits, rows, cols, q_out, positions, cos_sin, slot_mapping,
                          k_cache, v_cache, nq, nkv, head_dim, residual, eps)
    return q_out


# ---------------------------------------------------------------------------------
# fused decode layer GEMMs (csrc/kernels/skinny_pkr.hip)
# ---------------------------------------------------------------------------------

_PKR_EPI = {"store": 0, "silu": 1, "resid": 2}
# (nt, depth) instantiated for every epilogue; "silu" needs an even nt
PKR_CONFIGS = [(1, 2), (1, 4), (2, 2), (2, 3), (2, 4), (4, 2), (4, 3)]


def interleave_gate_up(w: torch.Tensor, nh: int) -> torch.Tensor:
    """[2I, K] gate rows then up rows -> the row order of the fused gate_up + SiLU
    kernel with nt = 2 * nh column tiles per workgroup: for each block of 16 * nh
    outputs, its gate rows then its up rows."""
    two_i, k = w.shape
    inter = two_i // 2
    r = 16 * nh
    assert inter % r == 0
    g = w[:inter].reshape(inter // r, r, k)
    u = w[inter:].reshape(inter // r, r, k)
    return torch.stack([g, u], dim=1).reshape(two_i, k)


def pkr_gemm(x, w_pk, epi: str = "store", out=None, ws=None, residual=None, tickets=None,
             splits: int = 1, nt: int = 2, depth: int = 3, norm: bool = False, eps: float = 0.0,
             wn: bool = False):
    """Ring-pipelined decode GEMM (M <= 64) on pack_weight() images.

    * ``store``: bf16 ``out`` (one split) or fp32 slabs [splits, M, N] in ``ws``.
    * ``silu``: w_pk packs interleave_gate_up(W_gu, nt // 2); returns h = silu(g) * u
      [M, N/2]; ``norm``: x rows RMS-normalised on the fly (norm weight folded into W).
    * ``resid``: ``residual`` += x w^T, split-K reduced inside the launch (``tickets``:
      zeroed int32, >= N / (16 nt), left zeroed).
    * ``wn``: wave-split-N layout for 33-64 rows (N % (64 nt) == 0): x fragments
      shared by the workgroup's 4 waves through L1."""
    if epi == "silu" and out is None:
        out = torch.empty(x.shape[0], w_pk.shape[0] // 2, dtype=x.dtype, device=x.device)
    native().pkr_gemm(x, w_pk, out, ws, residual, tickets, splits, nt, depth, _PKR_EPI[epi],
                      norm, eps, wn)
    return out


# ---------------------------------------------------------------------------------
# persistent post-attention decode block (csrc/kernels/decode_block.hip)
# ---------------------------------------------------------------------------------

def decode_block_plan(hidden: int, attn_dim: int, inter: int):
    """(o splits, down splits, gate_up tiles per workgroup, grid) when the block
    kernel covers this layer shape on the current device, else None."""
    if not native_available():
        return None
    return native().decode_block_plan(hidden, attn_dim, inter)


def decode_block_ws_floats(hidden: int, rows: int) -> int:
    """fp32 split-K slab floats the block kernel needs at ``rows`` rows."""
    return int(native().decode_block_ws_floats(hidden, rows))


def decode_block_ctl_words() -> int:
    return int(native().decode_block_ctl_words())


def decode_block(attn, residual, h, wo_pk, wgu_pk, wd_pk, ws, xg, ctl, eps: float, stamps=None):
    """One launch per layer after the attention: residual += attn Wo^T; h = silu(g) * u
    of rmsnorm(residual) Wgu^T (the norm weight folded into the interleaved packed
    gate_up image, the 1/rms applied in the epilogue); residual += h Wd^T.  ``h``
    [>= rows, I] bf16 scratch; ``ws`` / ``xg`` fp32 scratch; ``ctl`` int32 counters
    (zeroed, left zeroed; word 2 is a sticky give-up flag)."""
    native().decode_block(attn, residual, h, wo_pk, wgu_pk, wd_pk, ws, xg, ctl, eps, stamps)
    return residual
