"""Llama-3 decoder for the in-process engine (replaces the vLLM container the
reference talks to over HTTP: ``app/core/vllm_handler.py:53-62``).

Per layer:  fused add+RMSNorm (K2, HIP) -> QKV GEMM (K3, HIP
packed MFMA) -> RoPE + paged KV write (K4, HIP) -> prefill flash attention (K5,
HIP/MFMA) or paged MFMA decode attention (K6, HIP) -> O GEMM (K7) [+ RCCL
all-reduce under TP] -> fused add+RMSNorm -> gate_up GEMM (K8) -> SiLU-mul
(K9, HIP) -> down GEMM (K10) [+ all-reduce].  Only the last-token rows reach the
final norm and the LM head (K11), and the sampler (K12) consumes bf16 logits
directly.  The same code runs the CPU backend through the fp32 reference ops.
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import quant as Q
from ..ops import reference as ref
from ..parallel.comm import SINGLE, TPComm
from .config import ModelConfig
from . import weights as W

log = logging.getLogger(__name__)


@dataclasses.dataclass
class AttnMeta:
    """Per-step attention metadata (device tensors, int32).

    Rows ``[0, num_decode)`` are decode rows (one new token per sequence, paged
    split-K decode kernel); rows ``[num_decode, T)`` are prefill chunks (varlen
    MFMA prefill kernel).  A step may contain either or both (mixed batching).
    """
    positions: torch.Tensor          # [T]
    slot_mapping: torch.Tensor       # [T]
    logits_indices: torch.Tensor     # [B] rows that need logits (int64)
    num_decode: int = 0
    # decode rows
    dec_block_tables: Optional[torch.Tensor] = None   # [num_decode, max_blocks]
    dec_seq_lens: Optional[torch.Tensor] = None       # [num_decode]
    tmp_out: Optional[torch.Tensor] = None            # decode partials (ops.decode_workspace)
    tmp_ml: Optional[torch.Tensor] = None
    dec_counters: Optional[torch.Tensor] = None       # in-launch combine tickets (ops.decode_counters)
    # prefill rows
    block_tables: Optional[torch.Tensor] = None       # [P, max_blocks]
    seq_lens: Optional[torch.Tensor] = None           # [P] kv length after this step
    q_start_loc: Optional[torch.Tensor] = None        # [P+1], relative to row num_decode
    tile_info: Optional[torch.Tensor] = None          # [num_tiles*4] (ops.build_prefill_tiles)
    num_tiles: int = 0
    pf_part_o: Optional[torch.Tensor] = None          # split-KV prefill partials + combine list
    pf_part_ml: Optional[torch.Tensor] = None
    pf_combine: Optional[torch.Tensor] = None
    pf_num_combine: int = 0
    pf_num_partials: int = 0

    @property
    def is_prefill(self) -> bool:
        return self.num_decode == 0


@dataclasses.dataclass
class LayerWeights:
    wqkv: Optional[torch.Tensor]   # None when the projection is held as W4 only
    wo: Optional[torch.Tensor]
    wgu: Optional[torch.Tensor]
    wd: Optional[torch.Tensor]
    ln1: torch.Tensor
    ln2: torch.Tensor
    # the same weights in the MFMA-fragment image the decode GEMMs stream
    wqkv_pk: Optional[torch.Tensor] = None
    wo_pk: Optional[torch.Tensor] = None
    wgu_pk: Optional[torch.Tensor] = None
    wd_pk: Optional[torch.Tensor] = None
    # fused decode layer (skinny_pkr.hip): QKV / gate_up packed with the input norms
    # folded in (W diag(ln)), gate_up rows interleaved for the SiLU epilogue; o / down
    # share the packed images above when present
    fqkv: Optional[torch.Tensor] = None
    fo: Optional[torch.Tensor] = None
    fgu: Optional[torch.Tensor] = None
    fd: Optional[torch.Tensor] = None
    # W4A16 (AWQ) projections by name ("qkv", "o", "gu", "down"), GPU only
    q4: Optional[dict] = None


_ATTR = {"qkv": "wqkv", "o": "wo", "gu": "wgu", "down": "wd"}


# Decode GEMMs (<= 64 rows) on pre-packed weights (csrc/kernels/skinny_gemm.hip,
# "pk"/"xcp").  Per projection and row bucket: (nt, u, splits).  Chosen from
# cold-cache sweeps on MI355X (bench/gemm_sweep.py, us at M = 1 / 8 / 16 / 32 / 64;
# hipBLASLt on row-major weights, measured for reference in round 2, after "vs"):
#   qkv     9.8 / 10.3 / 11.1  vs 14-15
#   o       7.3 / 7.5 / 7.7 / 9.0 / 13.1 vs 14-15   split 2 -> slabs -> add+RMSNorm
#   gate_up 35 / 38 / 41 / 45            vs 55-66
#   down    18.6 / 19.3 / 20 / 22 / 28   vs 26-40   split 2-4 -> slabs -> add+RMSNorm
#   lm_head 148 / 161 / 174 / 184 / 197  vs 188-212
# Split-K partial sums stay fp32 in one workspace and are reduced inside the
# residual-add + RMSNorm that follows (row_rmsnorm from slabs): no extra kernel.
PACKED_ROWS = 64
# Batch-invariant mode (ENGINE_BATCH_INVARIANT): one (nt, splits) per projection at
# EVERY row count -- the xr decode kernel up to 64 rows, packed_gemm above -- so a
# row's sums run over the same K slices in the same order (k-steps ascending, fp32
# slabs summed 0..splits-1 by the consumer) whatever else is in the step.
INV_PLAN = {"qkv": (1, 2), "o": (1, 4), "gu": (2, 1), "down": (1, 4), "lm": (2, 1)}
_M_BUCKETS = (1, 8, 16, 32, 64)
PACKED_PLAN = {
    # qkv 32 / 64: split-K slabs reduced by slab_rope_kv (the bf16 image is the only
    # copy of the weights, so there is no hipBLASLt fallback)
    # 32 / 64 rows: "xc" with 8 splits (x chunk staged once per workgroup in LDS, 384
    # workgroups): qkv 14.7 vs 18.2 us, o 12.4 vs 13.1 us at 50-64 rows, engine A/B
    # 8.05 vs 8.22 ms/step (profiles/ab_decode_plan_xc8_r02.log)
    # 33-64 rows: "xr" (xc with the chunk loop pipelined: no drain between 512-wide
    # K chunks), so fewer splits pay: cold-cache us at 50 rows, xr vs the previous
    # plan (profiles/xr_vs_xc_decode_gemm_r02.log): qkv 14.6 (2 splits) vs 15.2
    # (xc, 8), o 10.9 (4) vs 13.1 (xc, 8), gate_up 44.7 with its own SiLU epilogue
    # vs 47.9 + 6.3 (xc 2 splits + slab_silu), down 25.3 vs 26.3 (pk), LM head
    # 181 vs ~195.  Fewer splits also shrink the slabs the next kernel re-reads.
    "qkv": {1: (1, -3, 1), 8: (2, -3, 1), 16: (2, -3, 1), 32: (2, -4, 8), 64: (1, -5, 2)},
    "o": {1: (1, -3, 2), 8: (2, -3, 2), 16: (2, -3, 2), 32: (2, -3, 2), 64: (1, -5, 4)},
    "gu": {1: (1, -3, 1), 8: (1, -3, 1), 16: (4, -3, 1), 32: (4, -3, 1), 64: (2, -6, 1)},
    # (at M = 64 the cold-cache sweep prefers down 2/-5/7 and LM head 1/-5/1, but in the
    # decode graph they measured 0.05 ms/step SLOWER: profiles/ab_sampler_plan_r02.log)
    "down": {1: (1, -3, 2), 8: (2, -3, 4), 16: (4, -3, 4), 32: (4, -3, 4), 64: (1, -5, 4)},
    "lm": {1: (1, -3, 1), 8: (2, -3, 1), 16: (4, -3, 1), 32: (1, -4, 1), 64: (2, -5, 1)},
}
# (33-64 rows, o / down on 8-wave workgroups with 8 splits -- one staged x chunk
# feeding twice the weight columns -- won the cold-cache sweep, o 9.8 vs 10.4 us, down
# 22.8 vs 25.3 us at 50 rows (profiles/xr8_sweep_r03.log), but lost in the decode graph,
# 7.66 vs 7.61 ms/step: the 8-split slabs cost the add+RMSNorm kernels more than the
# GEMMs save (profiles/ab_xr8_r03.log).  The kernel keeps the 8-wave form (u = -7 / -8)
# for plans that want it; the env switch is gone.)
MAX_SPLITS = 4


# Above PACKED_ROWS rows: packed_gemm.hip on the same image, (row limit, tile cfg,
# split-K) per projection from bench/pg_probe.py on MI355X vs hipBLASLt on row-major
# weights (profiles/packed_gemm_*_r02.log): split-K fills the chip at mixed-step
# sizes (80-256 rows: 0.8-1.7x hipBLASLt), whole tiles above.
# Soft-budgeted mixed steps land at <= 512 rows (entries re-checked at 300 / 400 /
# 512 rows: profiles/pg_probe_300_512_r02.log).  Up to 2047 rows the M = 1024
# measurements rule: split-K keeps o / down at 512 workgroups (whole tiles there:
# 80 workgroups on 256 CUs, 2-3x slower).
# 129-192 and 257-384 rows: the 192-row tiles (cfg 5 = 192x256, 6 = 192x128) pad the
# step to 192 / 384 MFMA rows instead of 256 / 512 -- profiles/pg_probe_192_r04.log:
# gate_up 54.8 vs 67.8 us at 145 rows, 81.4 vs 102.4 at 300, 88.2 vs 105.3 at 384;
# down 36.2 vs 43.7 / 54.3 vs 63.8 / 57.5 vs 66.3; LM head 233 vs 263 / 376 vs 463.
PG_PLAN = {
    "qkv": ((128, 1, 8), (192, 6, 4), (256, 2, 4), (384, 6, 2), (512, 2, 2), (2047, 0, 2),
            (1 << 30, 2, 1)),
    "o": ((128, 2, 8), (192, 6, 8), (256, 1, 8), (384, 6, 4), (512, 2, 4), (2047, 1, 2),
          (1 << 30, 0, 1)),
    "gu": ((128, 1, 2), (192, 6, 1), (256, 2, 1), (384, 5, 1), (1 << 30, 0, 1)),
    "down": ((128, 1, 16), (192, 6, 8), (256, 1, 8), (384, 5, 8), (512, 0, 8), (2047, 0, 4),
             (1 << 30, 3, 1)),
    "lm": ((128, 1, 1), (192, 5, 1), (256, 3, 1), (384, 5, 1), (1 << 30, 0, 1)),
}
PG_MAX_SLAB_ROWS = 2048
# hipBLASLt detours removed in round 5: unpacking the packed image into a row-major
# copy for the library from 2048 rows (FT_PG_BLAS_ROWS) measured neutral end to end
# (config 5 4,806 vs 4,820 tok/s, driver 5,672 vs 5,700: profiles/ab_pg_blas_rows_r05.log),
# and resident row-major copies for 257+ rows (FT_ROWMAJOR_COPIES) +1.2%, within the
# spread, for 10 GB (profiles/ab_rowmajor_copies_r03.log).  Every GEMM of the model
# runs the hand-written kernels on the packed image.


def pg_cfg(proj: str, rows: int, k: int) -> Tuple[int, int]:
    for lim, cfg, sp in PG_PLAN[proj]:
        if rows <= lim:
            break
    while sp > 1 and k % (64 * sp):
        sp //= 2
    return cfg, sp


def _cfg_fits(c, n: int, k: int) -> bool:
    nt, u, sp = c
    kq = {-4: 512, -5: 512 if nt == 2 else 256, -6: 512,
          -7: 512 if nt == 2 else 256, -8: 512}.get(u, 64)
    if u in (-6, -8) and (nt != 2 or sp != 1 or n % 32):
        return False
    return n % (16 * nt) == 0 and k % (kq * sp) == 0 and (u != -4 or n % 64 == 0)


def _overlay_packed_plan(spec: str):
    """FT_PACKED_PLAN='{"qkv": {"64": [4, -3, 2]}}' overlays PACKED_PLAN entries
    (A/B tuning on the GPU box without code edits); [] removes a bucket."""
    for proj, per in json.loads(spec).items():
        for b, c in per.items():
            if proj in PACKED_PLAN and int(b) in (1, 8, 16, 32, 64):
                if c:
                    PACKED_PLAN[proj][int(b)] = tuple(int(v) for v in c[:3])
                else:
                    PACKED_PLAN[proj].pop(int(b), None)


if os.environ.get("FT_PACKED_PLAN"):
    _overlay_packed_plan(os.environ["FT_PACKED_PLAN"])

# Fused decode layer (csrc/kernels/skinny_pkr.hip), <= FUSED_ROWS rows, bf16, TP=1:
# per layer four ring-pipelined packed GEMMs + RoPE/KV + attention, and no separate
# norm / SiLU / residual-add launches:
#   qkv   store -> split-K slabs; slab_rope_kv scales each row by its residual RMS
#   o     resid -> residual += attn Wo^T (split-K reduced inside the launch)
#   gu    silu + norm -> h = silu(g) * u of rmsnorm(residual) (ln2 folded into W)
#   down  resid -> residual += h Wd^T
# Per projection and row bucket: (nt, depth, splits, wn) -- wn: wave-split-N layout
# (33-64 rows).  fused_plan.json (written by bench/pkr_sweep.py --plan-out from
# cold-cache sweeps on MI355X) overrides these.
# Row limit of the fused layer (decode step, Llama-3-8B, MI355X): 8 sessions 2.3k vs
# 2.06k tok/s unfused, 32 sessions 4.52 vs 4.53 ms, 48 sessions 5.47 vs 5.54 ms; at
# 49-64 rows (four 16-row m-tiles) the ring kernels lose (50 sessions 6.2 vs 5.7 ms).
# Since gate_up at 33-64 rows runs as split-K slabs + slab_silu, the unfused layer
# also wins at 33-48 rows (40 sequences: 5.15 vs 5.45 ms/step), so the limit is 32.
FUSED_ROWS = int(os.environ.get("FT_FUSED_ROWS", "32"))
MAX_FUSED_SPLITS = 8
_FUSED_BUCKETS = (1, 8, 16, 32, 48, 64)
FUSED_PLAN = {
    "qkv": {1: (2, 3, 8, 0), 8: (2, 3, 8, 0), 16: (2, 3, 4, 0), 32: (2, 3, 2, 0),
            48: (4, 2, 8, 1), 64: (4, 2, 8, 1)},
    "o": {1: (1, 4, 1, 0), 8: (1, 4, 1, 0), 16: (1, 4, 1, 0), 32: (1, 4, 2, 0),
          48: (1, 2, 1, 0), 64: (1, 2, 1, 0)},
    "gu": {1: (2, 2, 1, 0), 8: (2, 4, 1, 0), 16: (2, 4, 1, 0), 32: (2, 4, 1, 0),
           48: (2, 2, 1, 1), 64: (2, 2, 1, 1)},
    "down": {1: (1, 4, 1, 0), 8: (1, 4, 1, 0), 16: (1, 4, 1, 0), 32: (1, 4, 2, 0),
             48: (4, 2, 4, 0), 64: (4, 2, 4, 0)},
}
_SILU_CONFIGS = ((2, 2), (2, 3), (2, 4), (4, 2), (4, 3))
# Persistent post-attention decode block (csrc/kernels/decode_block.hip), bf16, TP=1,
# BLOCK_MIN_ROWS..64 rows, OPT-IN (FT_DECODE_BLOCK=1): per layer the QKV xr GEMM on the
# raw residual (ln1 folded in), slab_rope_kv (applies the input RMS), the decode
# attention and ONE launch for o -> add -> RMSNorm -> gate_up+SiLU -> down -> add.
# Measured 96-98 us per layer against 86 us for the five launches it replaces at 50
# rows (profiles/decode_block_r06.log): each in-launch hand-off costs 5-10 us once the
# weight streams saturate HBM, kernel boundaries 1.2-1.9 us.  Never enabled where
# several processes share the device (its grid must be resident: one workgroup per CU).
BLOCK_ROWS = 64
BLOCK_MIN_ROWS = int(os.environ.get("FT_DECODE_BLOCK_MIN_ROWS", str(FUSED_ROWS + 1)))


def _decode_block_enabled() -> bool:
    if os.environ.get("FT_DECODE_BLOCK", "0").lower() not in ("1", "true", "on"):
        return False
    shared = (os.environ.get("FT_BENCH_SHARED_GPU", "0") == "1"
              or os.environ.get("ENGINE_KV_SIZING", "") == "own"
              or os.environ.get("ENGINE_TP_SHARE_DEVICE", "0").lower() in ("1", "true"))
    return not shared
# (Measured negatives, removed: the QKV projection with RoPE + the paged K/V write
# in its own epilogue -- 3.52 vs 3.25 ms per single-session decode step, the
# in-launch split-K seam costs more than the launch it saves
# (profiles/qkv_rope_ab_r04.log); and RoPE + the K/V write inside the decode
# attention launch -- 4.03 vs 3.27 ms single-session, 6.38 vs 6.23 ms at 50
# sessions: every attention wave rebuilding its q from the slabs puts two dependent
# memory round trips in front of its KV stream (profiles/rope_in_attention_ab_r04.log).)
_FUSED_PLAN_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fused_plan.json")


def load_fused_plan(path: str = _FUSED_PLAN_FILE):
    """Overlays a measured plan {proj: {bucket: [nt, depth, splits]}} on FUSED_PLAN."""
    if not os.path.exists(path):
        return
    with open(path) as f:
        plan = json.load(f)
    for proj, per in plan.items():
        ok = _SILU_CONFIGS if proj == "gu" else [tuple(c) for c in ops.PKR_CONFIGS]
        for b, c in per.items():
            c = tuple(int(v) for v in c[:4]) + (0,) * (4 - len(c[:4]))
            if proj in FUSED_PLAN and int(b) in _FUSED_BUCKETS and c[:2] in ok \
                    and 1 <= c[2] <= MAX_FUSED_SPLITS and c[3] in (0, 1):
                FUSED_PLAN[proj][int(b)] = c


load_fused_plan()


def fused_bucket(rows: int) -> int:
    return next(m for m in _FUSED_BUCKETS if m >= rows)


def fused_cfg(proj: str, rows: int, n: int, k: int, nt_fixed: Optional[int] = None):
    """(nt, depth, splits, wn) for one fused-layer GEMM: the plan entry, unless the
    shape rules it out (then one split, nt 1 if the columns do not tile, no wn)."""
    nt, depth, sp, wn = FUSED_PLAN[proj][fused_bucket(rows)]
    if nt_fixed is not None and nt != nt_fixed:  # gate_up: the packing fixes nt
        nt, depth = nt_fixed, 2
    if k % (64 * sp):
        sp = 1
    if n % (16 * nt):
        nt, depth = 1, 2
    wn = bool(wn) and rows > 32 and n % (64 * nt) == 0
    return nt, depth, sp, wn


def _fold_norm(w: torch.Tensor, ln: torch.Tensor) -> torch.Tensor:
    """W diag(ln): the RMSNorm weight moved onto the GEMM's K axis."""
    return (w.float() * ln.float()[None, :]).to(w.dtype)

# W4A16 decode GEMMs (csrc/kernels/w4a16.hip): (nt, splits, xr) per projection and
# row bucket.  <= 16 rows: the register kernel, from cold-cache sweeps on MI355X
# (bench/w4_sweep.py, us at M = 1 / 8 / 16; bf16 packed plan in brackets):
#   qkv   5.7 / 6.0 / 6.5   [9.8 / 10.3 / 11.1]
#   o     4.4 / 4.7 / 5.1   [7.3 / 7.5 / 7.7]
#   gu    15.2 / 14.9 / 16.7  [35 / 38 / 41]
#   down  9.2 / 8.5 / 9.1   [18.6 / 19.3 / 20]
# 17..64 rows: the x-in-LDS "xr" variant where it wins (bench/w4xr_sweep.py, us at
# M = 50 / 64, profiles/w4xr_sweep_r03.log): qkv 13.9 / 15.0 (register kernel 14.2 /
# 15.6), o 9.3 / 9.8 (10.8 / 11.7), gate_up with the SiLU epilogue on its interleaved
# image 40.1 / 41.2 (41.0 / 45.6 + silu_mul); down stays on the register kernel (20.1
# / 21.8 vs 23.4 / 24.3).  At 64 rows W4 is MFMA + dequant bound (the same MFMA work
# as bf16 on a quarter of the bytes): 83 vs 95 us per layer for the bf16 image.
# qkv, o and down leave split-K slabs: qkv's are reduced by the RoPE + KV-write
# kernel (slab_rope_kv), o's and down's by the fused add+RMSNorm.
W4_ROWS = 64
W4_PLAN = {
    "qkv": {1: (2, 8, 0), 8: (4, 2, 0), 16: (4, 2, 0), 32: (2, 4, 1), 64: (2, 4, 1)},
    "o": {1: (2, 8, 0), 8: (2, 8, 0), 16: (4, 8, 0), 32: (2, 8, 1), 64: (2, 8, 1)},
    "gu": {1: (4, 1, 0), 8: (4, 1, 0), 16: (4, 1, 0), 32: (2, 1, 1), 64: (2, 1, 1)},
    "down": {1: (4, 4, 0), 8: (4, 4, 0), 16: (4, 4, 0), 32: (4, 4, 0), 64: (4, 4, 0)},
}


# 49..64 rows: the "mh" kernel (w4a16.hip, xr 4 = weight ring 2 with two x chunks in
# flight, 5 = ring 3) where it wins, cold-cache us at 50 / 64 rows on MI355X
# (bench/w4mx_sweep.py, profiles/w4_mh_r06.log): qkv 12.2 / 12.7 (xr 13.9 / 14.6),
# o 8.8 / 9.4 (9.2 / 9.6), gate_up + SiLU 38.5 / 38.9 (40.0 / 41.2); down keeps the
# register kernel (19.7 vs 20.1).  At 33..48 rows the second row half is mostly
# padding and xr stays ahead (gate_up 31.3 vs 39.0 at 33 rows).
W4_PLAN_MH = {"qkv": (2, 4, 4), "o": (2, 8, 4), "gu": (2, 1, 5)}
W4_MH_MIN_ROWS = 49
# Llama-3-70B at TP=1 (>= 64 M-weight projections), 49..64 rows, cold-cache us at 50
# rows (profiles/w4_70b_sweep_r06.log): qkv mh at 8 splits 33.2 (4 splits 40.3), o the
# register kernel at 2 splits 22.7 (mh / 8: 25.6); gate_up (K 8192 > mh's K slice)
# stays on the xr SiLU entry, down on the register kernel.
W4_PLAN_WIDE = {"qkv": (2, 8, 4), "o": (4, 2, 0)}


def w4_cfg(proj: str, rows: int, n: int = 0, k: int = 0):
    """(nt, splits, xr) of a W4 decode GEMM.  With the shape given, an entry whose
    kernel cannot tile it (TP shards, Llama-3-70B's K 8192 gate_up / 28672 down for
    mh's 4096-wide K slices) falls back to the bucket plan, then to the register
    kernel at one split."""
    b = next(m for m in _M_BUCKETS if m >= rows)
    cands = [W4_PLAN[proj][b]]
    if rows >= W4_MH_MIN_ROWS and proj in W4_PLAN_MH:
        cands.insert(0, W4_PLAN_MH[proj])
    if rows >= W4_MH_MIN_ROWS and n * k >= WIDE_ELEMS and proj in W4_PLAN_WIDE:
        cands.insert(0, W4_PLAN_WIDE[proj])
    if not n:
        return cands[0]
    for c in cands:
        if w4_fits(c[2], c[0], c[1], n, k):
            return c
    return (1, 1, 0)


def w4_fits(xr: int, nt: int, sp: int, n: int, k: int) -> bool:
    """Whether the W4 decode kernel ``xr`` (0 register, 1 xr, 4 / 5 mh) tiles [n, k]
    at ``sp`` K splits (TP shards can break the plan's shapes)."""
    if xr in (4, 5):
        return n % 32 == 0 and k % (256 * sp) == 0 and k // sp <= 4096
    if xr:
        return n % (64 * nt) == 0 and k % (512 * sp) == 0
    return n % (16 * nt) == 0 and k % (128 * sp) == 0


# Projections of >= 64 M weights (Llama-3-70B at TP=1: qkv 10240 x 8192, o 8192 x 8192,
# down 8192 x 28672) at 33-64 rows: two column tiles per wave (qkv, down) or 8-wave
# workgroups (o), same splits -- cold-cache us at 50 rows, round 5
# (profiles/xr_sweep_70b_r05.log): qkv 35.3 vs 44.6, o 25.2 vs 28.3, down 77.9 vs 85.3.
# FT_WIDE_DECODE_PLAN=0 keeps the default plan for them.
PACKED_PLAN_WIDE = {"qkv": {64: (2, -5, 2)}, "o": {64: (1, -7, 4)}, "down": {64: (2, -5, 4)}}
WIDE_ELEMS = 64 << 20
WIDE_PLAN = os.environ.get("FT_WIDE_DECODE_PLAN", "1") != "0"


def packed_cfg(proj: str, rows: int, n: int = 0, k: int = 0):
    if rows > PACKED_ROWS:
        return None
    b = next(m for m in _M_BUCKETS if m >= rows)
    if WIDE_PLAN and n * k >= WIDE_ELEMS:
        c = PACKED_PLAN_WIDE.get(proj, {}).get(b)
        if c is not None:
            return c
    return PACKED_PLAN[proj].get(b)


def _packable(n: int, k: int, proj: str) -> bool:
    """Every configuration the plan may pick for this projection fits the shape."""
    for nt, u, sp in PACKED_PLAN[proj].values():
        kq = 512 if u == -4 else 64
        if n % (16 * nt) or k % (kq * sp) or n % 64:
            return False
    return True


class LlamaModel:
    def __init__(self, cfg: ModelConfig, device: torch.device, dtype: torch.dtype = torch.bfloat16,
                 comm: TPComm = SINGLE, max_model_len: int = 8192, quantization: Optional[str] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.comm = comm
        self.tp = comm.world_size
        self.rank = comm.rank
        self.nq, self.nkv = W.tp_heads(cfg, self.tp)
        self.d = cfg.head_dim
        self.scale = self.d ** -0.5
        self.vocab_shard = cfg.vocab_size // self.tp
        assert cfg.vocab_size % self.tp == 0
        self.max_model_len = max_model_len
        self.layers: List[LayerWeights] = []
        self.embed: Optional[torch.Tensor] = None
        self.norm: Optional[torch.Tensor] = None
        self.lm_head: Optional[torch.Tensor] = None
        self.cos_sin = ref.rope_cos_sin(self.d, max(max_model_len, 16) + 1, cfg.rope_theta,
                                        cfg.rope_scaling, device=self.device)
        self.lm_head_pk: Optional[torch.Tensor] = None
        self.ws: Optional[torch.Tensor] = None
        self.invariant = False          # set_batch_invariant()
        self.inv_plan: Dict[str, Tuple[int, int]] = {}
        self.use_packed = (self.device.type == "cuda" and dtype == torch.bfloat16
                           and os.environ.get("FT_PACKED_GEMM", "1") != "0")
        # "awq" / "w4": layer projections as W4A16 (group 128).  On the GPU only the
        # packed int4 image is kept; the CPU backend holds the dequantized weights.
        self.quant = (quantization or "").lower() or None
        if self.quant not in (None, "awq", "w4"):
            raise ValueError(f"unsupported quantization {quantization!r} (awq | w4)")
        self._w4_scratch: Optional[torch.Tensor] = None
        self.w4_gu_il = False     # W4 gate_up image interleaved in 16-row groups
        self.fused = False
        self.mark_at = None   # (layer, event): recorded as the forward reaches that layer
        self.gu_nt = 2
        self.gu_il = False        # gate_up image interleaved in groups of 16 (packed bf16)
        self.w4_slab: dict = {}   # W4 projections that leave split-K slabs
        self.tickets: Optional[torch.Tensor] = None
        self.block = False        # persistent post-attention decode block (_prepare_block)
        self.db_h = self.db_xg = self.db_ctl = None
        # TP: all-reduce + residual add + RMSNorm in one launch (FT_TP_FUSED_NORM=0: the
        # separate slab_store -> all-reduce -> add+RMSNorm launches, for A/B runs)
        self.tp_fused_norm = os.environ.get("FT_TP_FUSED_NORM", "1") != "0"

    # ------------------------------------------------------------------ weights
    def _set_layers(self, shards):
        self.layers = [LayerWeights(**{k: v.to(self.device, self.dtype) for k, v in s.items()})
                       for s in shards]

    def init_random(self, seed: int = 0, std: float = 0.02, consistent: Optional[bool] = None):
        """Random-init weights.  ``consistent`` (default: small models) draws the
        full unsharded tensors on the host from one seed and slices them, so TP=N
        equals TP=1 exactly; otherwise every shard is drawn on the device."""
        cfg = self.cfg
        on_device = False
        if consistent is None and os.environ.get("FT_CONSISTENT_INIT"):
            # TP-vs-TP=1 tests; "device": the full tensors are drawn by the device's own
            # generator (same seed -> same values in every process on the same device
            # kind), seconds instead of minutes for 70B-shaped layers on the host
            mode = os.environ["FT_CONSISTENT_INIT"]
            consistent = mode in ("1", "device")
            on_device = mode == "device" and self.device.type == "cuda"
        if consistent is None:
            consistent = cfg.num_params() < 2_000_000_000 and self.device.type == "cpu" or \
                cfg.num_params() < 300_000_000
        if consistent:
            g = torch.Generator(device=self.device if on_device else "cpu").manual_seed(seed)
            embed = (torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g, device=g.device)
                     * std).to(self.dtype)
            shards = []
            for li in range(cfg.num_layers):
                full = W.random_full_layer(cfg, g, std, self.dtype)
                shards.append(W.shard_full_layer(cfg, full, self.rank, self.tp))
            self._set_layers(shards)
            lm = embed if cfg.tie_word_embeddings else \
                (torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g, device=g.device)
                 * std).to(self.dtype)
            self.embed = embed.to(self.device)
            self.lm_head = W._shard_rows(lm, self.rank, self.tp).contiguous().to(self.device)
        else:
            self.layers = []
            for li in range(cfg.num_layers):
                s = W.random_layer_fast(cfg, self.rank, self.tp, li, seed, std, self.dtype, self.device)
                self.layers.append(LayerWeights(**s))
            g = torch.Generator(device=self.device)
            g.manual_seed(seed * 7 + 3)
            self.embed = torch.empty(cfg.vocab_size, cfg.hidden_size, dtype=self.dtype,
                                     device=self.device).normal_(0.0, std, generator=g)
            if cfg.tie_word_embeddings:
                self.lm_head = W._shard_rows(self.embed, self.rank, self.tp)
            else:
                self.lm_head = torch.empty(self.vocab_shard, cfg.hidden_size, dtype=self.dtype,
                                           device=self.device).normal_(0.0, std, generator=g)
        self.norm = torch.ones(cfg.hidden_size, dtype=self.dtype, device=self.device)
        self._quantize_layers()
        self._prepare_packed()
        return self

    def load_checkpoint(self, ckpt_dir: str):
        cfg = self.cfg
        idx = W.SafetensorsIndex(ckpt_dir)
        awq = W.is_awq_checkpoint(idx)
        if awq and self.quant is None:
            self.quant = "awq"
        shards = []
        for li in range(cfg.num_layers):
            if awq:
                shards.append(W.load_awq_layer_shard(cfg, idx, li, self.rank, self.tp))
            else:
                full = W.load_full_layer(idx, li, self.dtype)
                shards.append(W.shard_full_layer(cfg, full, self.rank, self.tp))
        if awq:
            self._set_w4_layers(shards)
        else:
            self._set_layers(shards)
        self.embed = idx.get("model.embed_tokens.weight").to(self.device, self.dtype)
        self.norm = idx.get("model.norm.weight").to(self.device, self.dtype)
        if cfg.tie_word_embeddings or not idx.has("lm_head.weight"):
            lm = self.embed
        else:
            lm = idx.get("lm_head.weight").to(self.dtype)
        self.lm_head = W._shard_rows(lm, self.rank, self.tp).contiguous().to(self.device)
        if not awq:  # AWQ layers arrive quantized
            self._quantize_layers()
        self._prepare_packed()
        return self

    # ------------------------------------------------------------------ W4A16
    def _install_w4(self, L: LayerWeights, proj: str, q, z, s):
        if self.device.type == "cuda":
            if L.q4 is None:
                L.q4 = {}
            if proj == "gu" and q.shape[0] % 32 == 0:
                # gate/up rows interleaved in 16-row groups (quantization is per row, so
                # the permutation commutes with it): the W4 xr kernel's SiLU epilogue
                # pairs a gate tile with its up tile; every other path un-interleaves
                # through silu_mul(interleaved=True)
                q, z, s = (ops.interleave_gate_up(t, 1) for t in (q, z, s))
                self.w4_gu_il = True
            L.q4[proj] = Q.pack_w4(q.to(self.device), z.to(self.device), s.to(self.device))
            setattr(L, _ATTR[proj], None)
        else:  # CPU reference backend: the dequantized weight
            setattr(L, _ATTR[proj], Q.dequantize_w4(q, z, s).to(self.dtype))

    def _quantize_layers(self):
        """Round-to-nearest W4 of bf16 layer weights (random init or a bf16 checkpoint
        with ``quantization='w4'``); AWQ checkpoints arrive quantized."""
        if self.quant is None:
            return
        for L in self.layers:
            for proj, attr in _ATTR.items():
                w = getattr(L, attr)
                if w is None:
                    continue
                # from the bf16 values on every backend, so the CPU reference and the
                # GPU hold the same quantized weights
                q, z, sc = Q.quantize_w4(w.to(torch.bfloat16))
                self._install_w4(L, proj, q, z, sc)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)  # free the bf16 copies as we go

    def _set_w4_layers(self, shards):
        self.layers = []
        for sh in shards:
            L = LayerWeights(wqkv=None, wo=None, wgu=None, wd=None,
                             ln1=sh["ln1"].to(self.device, self.dtype),
                             ln2=sh["ln2"].to(self.device, self.dtype))
            for proj, attr in _ATTR.items():
                self._install_w4(L, proj, *sh[attr])
            self.layers.append(L)

    def _w4_prefill_dense(self, proj: str, dense: torch.Tensor) -> Optional[torch.Tensor]:
        """The dequantized weight as packed_gemm.hip wants it: gate_up in the 16-row
        interleave its SiLU epilogue pairs (the int4 image has it only when its row
        count allowed: _install_w4), None when the shape cannot be packed."""
        n, k = dense.shape
        if proj == "gu" and not self.w4_gu_il:
            if (n // 2) % 16:
                return None
            dense = ops.interleave_gate_up(dense, 1)
        if n % 16 or k % 64:
            return None
        return dense

    def _w4_packed(self, w: "Q.W4Weight", proj: str) -> Optional[torch.Tensor]:
        """A W4 projection dequantized and re-laid out into the packed image, in two
        shared scratches (prefill-size steps when the resident prefill image is off);
        None when the shape cannot be packed (the caller runs the dense fallback)."""
        need = w.n * w.k
        if w.n % 16 or w.k % 64 or (proj == "gu" and not self.w4_gu_il and (w.n // 2) % 16):
            return None
        if self._w4_scratch is None or self._w4_scratch.shape[1] < need:
            big = max(q.n * q.k for L in self.layers for q in (L.q4 or {}).values())
            self._w4_scratch = torch.empty(2, max(need, big), dtype=self.dtype, device=self.device)
        dense = Q.w4_dequant(w, out=self._w4_scratch[0, :need].view(w.n, w.k))
        dense = self._w4_prefill_dense(proj, dense)
        out = self._w4_scratch[1, :need]
        n, k = w.n, w.k
        out.view(n // 16, k // 64, 2, 4, 16, 8).copy_(
            dense.view(n // 16, 16, k // 64, 4, 2, 8).permute(0, 2, 4, 3, 1, 5))
        return out.view(n, k)

    def _prepare_w4_prefill(self):
        """W4A16 prefill image: every W4 projection dequantized ONCE into the packed
        bf16 layout (gate_up keeps the W4 image's 16-row interleave, which is the
        SiLU epilogue's), so steps above W4_ROWS rows run packed_gemm.hip on it
        instead of dequantizing every layer's weight into a scratch and calling
        hipBLASLt on every mixed step (15 GB written and read again per step for an
        8B model).  Decode steps keep streaming the int4 image.  FT_W4_PREFILL_IMAGE:
        auto (default: when a quarter of device memory stays free for the KV cache
        after the bf16 image -- 8B: 14 GB of 288; 70B at TP=1: 140 GB next to 35 GB of
        int4, 50 sessions 1,006 -> 1,386 tok/s, p50 TTFT 449 -> 165 ms,
        profiles/bench_70b_awq_image_s50_r06.log), 1, 0 (int4 only: the least memory,
        prefill-size steps dequantize per projection)."""
        mode = os.environ.get("FT_W4_PREFILL_IMAGE", "auto")
        if self.quant is None or mode == "0" or self.device.type != "cuda" or not self.layers:
            return
        qs = [(L, p, L.q4[p]) for L in self.layers for p in _ATTR if L.q4 and p in L.q4]
        if not qs:
            return
        nbytes = sum(q.n * q.k * 2 for _, _, q in qs)
        if mode != "1":
            free, total = torch.cuda.mem_get_info(self.device)
            if free - nbytes < 0.25 * total:
                return
        for L, p, q in qs:
            dense = self._w4_prefill_dense(p, Q.w4_dequant(q))
            if dense is not None:   # else packed per step (_w4_packed) or the dense fallback
                setattr(L, _ATTR[p] + "_pk", ops.pack_weight(dense))
        log.info("W4A16 prefill image (dequantized, packed bf16): %.1f GB", nbytes / 1e9)

    def _prepare_packed(self):
        """ONE weight image on the GPU (bf16): every layer projection and the LM head
        are re-laid out into the MFMA-fragment image the decode kernels stream
        (ops.pack_weight) and the row-major originals are dropped; prefill and large
        batches run packed_gemm.hip on the same bytes.  The input RMSNorm weights are
        folded into the QKV / gate_up images (W diag(ln)) -- the GPU norms then run
        with unit weights -- and gate_up is interleaved in groups of 16 rows so the
        fused SiLU epilogues see gate and up side by side.  Resident weights = the
        model size (+ the embedding table when it is not tied)."""
        if not self.use_packed or not self.layers:
            return
        cfg = self.cfg
        H = cfg.hidden_size
        fold = self.quant is None
        one = torch.ones(H, dtype=self.dtype, device=self.device)
        for L in self.layers:
            if L.wqkv is not None:
                w = _fold_norm(L.wqkv, L.ln1) if fold else L.wqkv
                L.wqkv_pk, L.wqkv = ops.pack_weight(w), None
            if L.wo is not None:
                L.wo_pk, L.wo = ops.pack_weight(L.wo), None
            if L.wgu is not None:
                w = _fold_norm(L.wgu, L.ln2) if fold else L.wgu
                L.wgu_pk, L.wgu = ops.pack_weight(ops.interleave_gate_up(w, 1)), None
            if L.wd is not None:
                L.wd_pk, L.wd = ops.pack_weight(L.wd), None
            if fold:
                L.ln1 = L.ln2 = one
        self._prepare_w4_prefill()
        # gate_up split-K slabs come from a 16-row-interleaved image: the packed bf16 one,
        # or (W4) the dequantized image, interleaved when the int4 image is not
        # (_w4_prefill_dense)
        self.gu_il = True
        if self.lm_head is not None:
            self.lm_head_pk = ops.pack_weight(self.lm_head)
            self.lm_head = None
        # split-K slab workspace: the largest [splits, rows, N] any plan may write
        L0 = self.layers[0]
        ns = {"qkv": (self.nq + 2 * self.nkv) * self.d, "o": H,
              "gu": 2 * cfg.intermediate_size // self.tp, "down": H}
        need = MAX_SPLITS * PACKED_ROWS * H
        for proj, n in ns.items():
            need = max(need, max(sp * b * n for b, (_, _, sp) in PACKED_PLAN[proj].items()))
            need = max(need, max((sp * min(lim, PG_MAX_SLAB_ROWS) * n
                                  for lim, _, sp in PG_PLAN[proj] if sp > 1), default=0))
        slab_w4 = self.tp == 1 and H % 2048 == 0
        for proj in ("qkv", "o", "down"):  # W4: the slab path depends on the shape rules only
            q = L0.q4.get(proj) if L0.q4 else None
            if q is None:
                continue
            self.w4_slab[proj] = slab_w4 and all(
                q.k % ((512 if xr else 128) * sp) == 0 and q.n % ((64 if xr else 16) * nt) == 0
                for nt, sp, xr in W4_PLAN[proj].values())
            if self.w4_slab[proj]:
                need = max(need, max(sp * b * q.n for b, (_, sp, _) in W4_PLAN[proj].items()))
        self.ws = torch.empty(need, dtype=torch.float32, device=self.device)
        # in-launch split-K tickets (fused ring layer): zeroed,
        # every launch leaves them zeroed
        self.tickets = torch.zeros(max(4096, H // 16), dtype=torch.int32, device=self.device)
        torch.cuda.empty_cache()
        self._prepare_fused()
        self._prepare_block()

    def _prepare_fused(self):
        """The fused decode layer (<= FUSED_ROWS rows) streams the same images: QKV /
        gate_up already carry ln1 / ln2 and gate_up is interleaved for nt = 2."""
        self.fused = False
        cfg = self.cfg
        H, I = cfg.hidden_size, cfg.intermediate_size
        nqkv = (self.nq + 2 * self.nkv) * self.d
        self.gu_nt = 2
        L0 = self.layers[0]
        if (self.quant or self.tp != 1 or os.environ.get("FT_FUSED_DECODE", "1") == "0"
                or L0.wqkv_pk is None or L0.wgu_pk is None or H % 64 or I % 64 or nqkv % 16):
            return
        for L in self.layers:
            L.fqkv, L.fo, L.fgu, L.fd = L.wqkv_pk, L.wo_pk, L.wgu_pk, L.wd_pk
        need = MAX_FUSED_SPLITS * FUSED_ROWS * max(nqkv, H)
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.float32, device=self.device)
        if self.tickets is None:
            self.tickets = torch.zeros(max(4096, H // 16), dtype=torch.int32, device=self.device)
        self.fused = True

    def _prepare_block(self):
        """Scratch and plan of the persistent decode block: it streams the same packed
        images (o, gate_up with ln2 folded and 16-row interleave, down)."""
        self.block = False
        cfg = self.cfg
        H, I = cfg.hidden_size, cfg.intermediate_size
        L0 = self.layers[0]
        if (self.quant or self.tp != 1 or not _decode_block_enabled() or L0.wo_pk is None
                or L0.wgu_pk is None or L0.wd_pk is None or L0.wqkv_pk is None):
            return
        plan = ops.decode_block_plan(H, self.nq * self.d, I)
        if plan is None:
            return
        so, sd, tpw, grid = plan
        need = ops.decode_block_ws_floats(H, BLOCK_ROWS)
        nqkv = (self.nq + 2 * self.nkv) * self.d
        need = max(need, MAX_SPLITS * BLOCK_ROWS * nqkv)
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.float32, device=self.device)
        self.db_h = torch.empty(BLOCK_ROWS, I, dtype=self.dtype, device=self.device)
        self.db_xg = torch.empty((grid // 2) * 2 * 4 * 256, dtype=torch.float32, device=self.device)
        self.db_ctl = torch.zeros(ops.decode_block_ctl_words(), dtype=torch.int32, device=self.device)
        self.block = True
        log.info("decode block: down splits %d, <= %d gate/up pairs per workgroup, grid %d",
                 sd, tpw, grid)

    def block_fault(self) -> bool:
        """True (and the block path switched off, its counters re-armed) if a decode
        block launch gave up waiting at a grid barrier (sticky word ctl[2])."""
        if self.db_ctl is None:
            return False
        if int(self.db_ctl[2].item()) == 0:
            return False
        log.error("decode block gave up at a grid barrier (error word %d): falling back "
                  "to the unfused decode layer", int(self.db_ctl[2].item()))
        torch.cuda.synchronize(self.device)
        self.db_ctl.zero_()
        self.block = False
        return True

    def resident_weight_bytes(self) -> int:
        """Bytes of weights held on the device (every layer tensor, embedding, head)."""
        seen, total = set(), 0

        def add(t):
            nonlocal total
            if isinstance(t, torch.Tensor) and t.device.type == self.device.type and \
                    t.data_ptr() not in seen:
                seen.add(t.data_ptr())
                total += t.numel() * t.element_size()
        for L in self.layers:
            for f in dataclasses.fields(L):
                v = getattr(L, f.name)
                if isinstance(v, dict):   # W4 projections / row-major copies
                    for q in v.values():
                        if isinstance(q, torch.Tensor):
                            add(q)
                            continue
                        for t in vars(q).values():
                            add(t)
                else:
                    add(v)
        for t in (self.embed, self.norm, self.lm_head, self.lm_head_pk):
            add(t)
        return total

    def set_batch_invariant(self, max_rows: int):
        """Batch-invariant numerics: INV_PLAN GEMMs at every row count, no fused decode
        layer, fixed-piece decode attention and per-row prefill rescales (the caller
        plans prefill with ops.build_prefill_tiles(fixed_chunk=...)).  A sequence's
        tokens then do not depend on what else shares its steps."""
        if self.tp != 1 or self.quant:
            raise ValueError("batch-invariant mode needs TP=1 and bf16 weights")
        self.fused = False
        self.invariant = True
        if self.layers[0].wqkv_pk is None:   # CPU / row-major reference path
            return
        nqkv = (self.nq + 2 * self.nkv) * self.d
        shapes = {"qkv": (nqkv, self.cfg.hidden_size), "o": (self.cfg.hidden_size, self.nq * self.d),
                  "gu": (2 * self.cfg.intermediate_size, self.cfg.hidden_size),
                  "down": (self.cfg.hidden_size, self.cfg.intermediate_size)}
        need = 0
        self.inv_plan = {"lm": INV_PLAN["lm"]}
        for proj, (n, k) in shapes.items():
            nt, sp = INV_PLAN[proj]
            kc = 512 if nt == 2 else 256
            while sp > 1 and k % (kc * sp):   # fewer slices for a K the plan does not divide
                sp //= 2
            if n % (16 * nt) or k % (kc * sp) or (proj == "gu" and (nt != 2 or sp != 1)):
                raise ValueError(f"batch-invariant plan does not fit {proj} {n}x{k}")
            self.inv_plan[proj] = (nt, sp)
            if sp > 1:
                need = max(need, sp * max_rows * n)
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.float32, device=self.device)

    def _packed_invariant(self, x: torch.Tensor, wp: torch.Tensor, proj: str):
        rows = x.shape[0]
        n, k = wp.shape
        nt, sp = self.inv_plan[proj]
        gu = proj == "gu"
        if sp > 1 and sp * rows * n > self.ws.numel():
            raise RuntimeError(f"batch-invariant workspace too small for {rows} rows")
        if rows <= PACKED_ROWS:
            u = -6 if gu else -5
            if sp > 1:
                ops.skinny_gemm(x, wp, ws=self.ws, splits=sp, nt=nt, u=u)
                return sp, None
            return 0, ops.skinny_gemm(x, wp, splits=1, nt=nt, u=u)
        cfg = pg_cfg(proj, rows, k)[0]
        if sp > 1:
            ops.packed_gemm(x, wp, ws=self.ws, splits=sp, epi="slab", cfg=cfg)
            return sp, None
        return 0, ops.packed_gemm(x, wp, epi="silu" if gu else "store", cfg=cfg)

    # ------------------------------------------------------------------ projections
    def _tp_fused(self, rows: int) -> bool:
        """TP decode-size steps: the row-parallel o / down outputs go through ONE
        launch -- custom all-reduce + residual add + RMSNorm (custom_ar.hip
        ar_add_rmsnorm_kernel) -- straight from their split-K slabs."""
        return (self.tp > 1 and self.tp_fused_norm
                and self.comm.fused_norm_ok(rows, self.cfg.hidden_size, self.device.type))

    def _tp_slabs(self, rows: int) -> bool:
        """TP steps of the fused path's shape: o / down leave split-K slabs whether
        the fused launch or the fallback (slab_store -> all-reduce -> add+norm) consumes
        them, so a group that fell back to RCCL reproduces the fused path's bits."""
        return (self.tp > 1 and self.tp_fused_norm
                and self.comm.fused_norm_shape(rows, self.cfg.hidden_size, self.device.type))

    def _slab_ok(self, proj: str, rows: int = 0) -> bool:
        """May this projection leave split-K fp32 slabs for its consumer?  qkv ->
        slab_rope_kv, gate_up -> slab_silu (both rank-local); o / down -> the
        residual add + RMSNorm (TP=1), or the fused all-reduce + add + RMSNorm
        (TP, custom collectives on); both need hidden % 2048."""
        if proj in ("qkv", "gu"):
            return True
        return self.cfg.hidden_size % 2048 == 0 and (self.tp == 1 or self._tp_slabs(rows))

    def _tp_add_norm(self, out, residual, weight, eps, t, splits, y, fused):
        """residual += all-reduce(partial); out = rmsnorm(residual) * weight, the
        partial being ``splits`` fp32 slabs in self.ws or the bf16 block y."""
        if fused:
            self.comm.all_reduce_add_rmsnorm(out, residual, weight, eps, t,
                                             ws=self.ws if splits else None, splits=splits,
                                             x=None if splits else y)
            return out
        if splits:
            y = torch.empty(t, self.cfg.hidden_size, dtype=self.dtype, device=self.device)
            ops.slab_store(self.ws, splits, t, y.shape[1], y)
        self.comm.all_reduce(y)
        ops.fused_add_rmsnorm(y, residual, weight, eps)
        return y

    def _lin(self, x: torch.Tensor, L: LayerWeights, proj: str) -> Tuple[int, Optional[torch.Tensor]]:
        """One layer projection y = x W^T.  Returns (splits, None) when the result
        is left as ``splits`` fp32 slabs in self.ws for the fused consumer, else
        (0, y).  For "gu" y is already h = silu(gate) * up."""
        rows = x.shape[0]
        q = L.q4.get(proj) if L.q4 else None
        if q is not None:  # W4A16
            il = proj == "gu" and self.w4_gu_il
            if rows <= W4_ROWS:
                nt, sp, xr = w4_cfg(proj, rows, q.n, q.k)
                if il and xr and nt == 2 and sp == 1 and q.n % (32 if xr in (4, 5) else 128) == 0:
                    return 0, Q.w4_gemm(x, q, nt=2, xr=xr, silu=True)
                if self.ws is not None and self.w4_slab.get(proj):
                    Q.w4_gemm(x, q, ws=self.ws, splits=sp, nt=nt, xr=xr)
                    return sp, None
                y = Q.w4_gemm(x, q, nt=nt, xr=xr)
            else:
                # the dequantized prefill image (_prepare_w4_prefill), or this
                # projection dequantized and packed into a scratch when it is off
                wp = getattr(L, _ATTR[proj] + "_pk")
                if wp is None:
                    wp = self._w4_packed(q, proj)
                if wp is not None:
                    return self._packed(x, wp, proj)
                # a shard shape packed_gemm cannot tile: the dequantized weight, dense
                y = F.linear(x, Q.w4_dequant(q))
            return 0, (ops.silu_mul(y, interleaved=il) if proj == "gu" else y)
        attr = _ATTR[proj]
        wp = getattr(L, attr + "_pk")
        if wp is None:  # row-major weights: CPU backend, or FT_PACKED_GEMM=0
            y = F.linear(x, getattr(L, attr))
            return 0, (ops.silu_mul(y) if proj == "gu" else y)
        return self._packed(x, wp, proj)

    def _packed(self, x: torch.Tensor, wp: torch.Tensor, proj: str) -> Tuple[int, Optional[torch.Tensor]]:
        """y = x W^T on the packed image: the decode kernels up to PACKED_ROWS rows
        (skinny_gemm.hip), the tiled MFMA GEMM above (packed_gemm.hip)."""
        if self.invariant:
            return self._packed_invariant(x, wp, proj)
        rows = x.shape[0]
        n, k = wp.shape
        gu = proj == "gu"
        slab_ok = self._slab_ok(proj, rows) and self.ws is not None
        c = packed_cfg(proj, rows, n, k) if proj in PACKED_PLAN else None
        while c is not None and c[2] > 1 and not _cfg_fits(c, n, k):
            c = (c[0], c[1], c[2] // 2)   # a K the plan's split does not divide (TP shards)
        if c is not None and _cfg_fits(c, n, k):
            nt, u, sp = c
            if sp > 1 and not (slab_ok and sp * rows * n <= self.ws.numel()):
                sp = 1
            if sp > 1:
                ops.skinny_gemm(x, wp, ws=self.ws, splits=sp, nt=nt, u=u)
                return sp, None
            y = ops.skinny_gemm(x, wp, splits=1, nt=nt, u=u)
            if u in (-6, -8):  # the xr kernel's own SiLU epilogue: y is already h
                return 0, y
            return 0, (ops.silu_mul(y, interleaved=True) if gu else y)
        cfg, sp = pg_cfg(proj, rows, k)
        if sp > 1 and (self.ws is None or sp * rows * n > self.ws.numel()):
            sp = 1
        if sp > 1:
            ops.packed_gemm(x, wp, ws=self.ws, splits=sp, epi="slab", cfg=cfg)
            if slab_ok:
                return sp, None
            y = torch.empty(rows, n, dtype=x.dtype, device=x.device)  # TP / odd hidden
            ops.slab_store(self.ws, sp, rows, n, y)
            return 0, y
        if gu:
            return 0, ops.packed_gemm(x, wp, epi="silu", cfg=cfg)
        return 0, ops.packed_gemm(x, wp, cfg=cfg)

    # ------------------------------------------------------------------ KV cache
    def kv_cache_shape(self, num_blocks: int, block_size: int) -> Tuple[int, ...]:
        """K cache shape; the V cache holds the same blocks transposed
        ([num_blocks, nkv, D, block_size]) so both MFMA operands of the attention
        kernels load straight from HBM (csrc/kernels/attn_decode.hip)."""
        return (num_blocks, self.nkv, block_size, self.d)

    def v_cache_shape(self, num_blocks: int, block_size: int) -> Tuple[int, ...]:
        return (num_blocks, self.nkv, self.d, block_size)

    def allocate_kv_cache(self, num_blocks: int, block_size: int, dtype=None):
        """[(K, V)] per layer in ``dtype`` (default: the compute dtype; fp8 =
        torch.float8_e4m3fn, written and read by the same kernels' KV8 paths)."""
        ks = self.kv_cache_shape(num_blocks, block_size)
        vs = self.v_cache_shape(num_blocks, block_size)
        dt = dtype or self.dtype
        return [(torch.zeros(ks, dtype=dt, device=self.device),
                 torch.zeros(vs, dtype=dt, device=self.device))
                for _ in range(self.cfg.num_layers)]

    # ------------------------------------------------------------------ forward
    def _attention(self, qkv: torch.Tensor, meta: AttnMeta, kc, vc) -> torch.Tensor:
        """Decode rows through the paged split-K kernel, prefill rows through the
        varlen MFMA kernel; q is read from the RoPE'd qkv rows."""
        t = qkv.shape[0]
        nq, nkv, d = self.nq, self.nkv, self.d
        attn = torch.empty(t, nq * d, dtype=qkv.dtype, device=qkv.device)
        nd = meta.num_decode
        if nd > 0:
            ops.decode_attention(attn[:nd], qkv[:nd], kc, vc, meta.dec_block_tables,
                                 meta.dec_seq_lens, meta.tmp_out, meta.tmp_ml, nq, nkv, d,
                                 self.scale, counters=meta.dec_counters,
                                 piece=ops.DECODE_INV_PIECE if self.invariant else 0)
        if t > nd:
            ops.prefill_attention(attn[nd:], qkv[nd:], kc, vc, meta.block_tables, meta.seq_lens,
                                  meta.q_start_loc, meta.tile_info, meta.num_tiles, nq, nkv, d,
                                  self.scale, meta.pf_part_o, meta.pf_part_ml, meta.pf_combine,
                                  meta.pf_num_combine, meta.pf_num_partials,
                                  invariant=self.invariant)
        return attn

    def _forward_fused(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """The fused decode layer (FUSED_PLAN): the residual stream is the GEMM input
        and the in-place output; every norm rides in a GEMM or the RoPE kernel."""
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        nq, nkv, d = self.nq, self.nkv, self.d
        t = input_ids.shape[0]
        H, I = cfg.hidden_size, cfg.intermediate_size
        nqkv = (nq + 2 * nkv) * d
        residual = self.embed.index_select(0, input_ids)
        cq = fused_cfg("qkv", t, nqkv, H)
        co = fused_cfg("o", t, H, nq * d)
        cg = fused_cfg("gu", t, 2 * I, H, nt_fixed=self.gu_nt)
        cd = fused_cfg("down", t, H, I)
        ws, tk = self.ws, self.tickets
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            qkv = torch.empty(t, nqkv, dtype=self.dtype, device=self.device)
            nt, dp, sp, wn = cq
            ops.pkr_gemm(residual, L.fqkv, "store", ws=ws, splits=sp, nt=nt, depth=dp, wn=wn)
            ops.slab_rope_kv(ws, sp, t, nqkv, qkv, meta.positions, self.cos_sin,
                             meta.slot_mapping, kc, vc, nq, nkv, d, residual=residual, eps=eps)
            attn = self._attention(qkv, meta, kc, vc)
            nt, dp, sp, wn = co
            ops.pkr_gemm(attn, L.fo, "resid", residual=residual, ws=ws, tickets=tk, splits=sp,
                         nt=nt, depth=dp, wn=wn)
            nt, dp, _, wn = cg
            h = ops.pkr_gemm(residual, L.fgu, "silu", nt=nt, depth=dp, norm=True, eps=eps, wn=wn)
            nt, dp, sp, wn = cd
            ops.pkr_gemm(h, L.fd, "resid", residual=residual, ws=ws, tickets=tk, splits=sp,
                         nt=nt, depth=dp, wn=wn)
        idx = meta.logits_indices
        rows = residual.index_select(0, idx) if idx.numel() != t else residual
        if rows.shape[0] == 0:
            return rows
        return ops.rmsnorm(rows, self.norm, eps)

    def _forward_block(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Decode rows through the persistent post-attention block: per layer the QKV
        GEMM on the raw residual (split-K slabs), slab_rope_kv (input RMS from the
        residual row, RoPE, paged K/V write), the decode attention, and ONE
        decode_block launch that leaves the next layer's residual."""
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        nq, nkv, d = self.nq, self.nkv, self.d
        t = input_ids.shape[0]
        H = cfg.hidden_size
        nqkv = (nq + 2 * nkv) * d
        nt, u, sp = packed_cfg("qkv", t, nqkv, H)
        if sp == 1:
            sp = 2   # slab_rope_kv reduces split-K slabs
        while sp > 1 and not _cfg_fits((nt, u, sp), nqkv, H):
            sp //= 2
        residual = self.embed.index_select(0, input_ids)
        mark = self.mark_at
        for li, L in enumerate(self.layers):
            if mark is not None and li == mark[0]:   # progress event (engine mixed chain)
                mark[1].record()
            kc, vc = kv_caches[li]
            qkv = torch.empty(t, nqkv, dtype=self.dtype, device=self.device)
            ops.skinny_gemm(residual, L.wqkv_pk, ws=self.ws, splits=sp, nt=nt, u=u)
            ops.slab_rope_kv(self.ws, sp, t, nqkv, qkv, meta.positions, self.cos_sin,
                             meta.slot_mapping, kc, vc, nq, nkv, d, residual=residual, eps=eps)
            attn = self._attention(qkv, meta, kc, vc)
            ops.decode_block(attn, residual, self.db_h, L.wo_pk, L.wgu_pk, L.wd_pk, self.ws,
                             self.db_xg, self.db_ctl, eps)
        idx = meta.logits_indices
        rows = residual.index_select(0, idx) if idx.numel() != t else residual
        if rows.shape[0] == 0:
            return rows
        return ops.rmsnorm(rows, self.norm, eps)

    def forward(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Returns the final-normed hidden rows at ``meta.logits_indices``."""
        t = input_ids.shape[0]
        if self.block and not self.invariant and BLOCK_MIN_ROWS <= t <= BLOCK_ROWS:
            return self._forward_block(input_ids, meta, kv_caches)
        if self.fused and input_ids.shape[0] <= FUSED_ROWS:
            return self._forward_fused(input_ids, meta, kv_caches)
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        nq, nkv, d = self.nq, self.nkv, self.d
        t = input_ids.shape[0]
        H = cfg.hidden_size
        residual = None
        x = None
        slab = 0  # >0: the previous down projection left that many fp32 slabs in self.ws
        # TP at decode sizes: o / down partials (slabs or bf16) are all-reduced inside
        # the next norm's launch; `pend` holds the last down's (splits, bf16 partial)
        tps = self._tp_slabs(t)
        tpf = tps and self._tp_fused(t)
        pend = None
        mark = self.mark_at
        for li, L in enumerate(self.layers):
            if mark is not None and li == mark[0]:   # progress event (engine mixed chain)
                mark[1].record()
            if residual is None:
                x, residual = ops.embed_rmsnorm(input_ids, self.embed, L.ln1, eps)  # K1 + K2
            elif pend is not None:   # residual += all-reduce(down partial); x = rmsnorm * ln1
                x = torch.empty(t, H, dtype=self.dtype, device=self.device) if tpf else None
                x = self._tp_add_norm(x, residual, L.ln1, eps, t, pend[0], pend[1], tpf)
                pend = None
            elif slab:  # residual += sum(slabs); x = rmsnorm(residual) * ln1
                x = torch.empty(t, H, dtype=self.dtype, device=self.device)
                ops.row_rmsnorm(x, L.ln1, eps, t, ws=self.ws, splits=slab, residual=residual)
            else:
                ops.fused_add_rmsnorm(x, residual, L.ln1, eps)
            kc, vc = kv_caches[li]
            sq, qkv = self._lin(x, L, "qkv")
            if sq:  # split-K slabs -> RoPE'd q and the paged K/V write in one kernel
                qkv = torch.empty(t, (nq + 2 * nkv) * d, dtype=self.dtype, device=self.device)
                ops.slab_rope_kv(self.ws, sq, t, qkv.shape[1], qkv, meta.positions, self.cos_sin,
                                 meta.slot_mapping, kc, vc, nq, nkv, d)
            else:
                ops.rope_kv_write(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc,
                                  nq, nkv, d)
            attn = self._attention(qkv, meta, kc, vc)
            so, y = self._lin(attn, L, "o")
            if tps:
                x = torch.empty(t, H, dtype=self.dtype, device=self.device) if tpf else None
                x = self._tp_add_norm(x, residual, L.ln2, eps, t, so, y, tpf)
            elif so:
                x = torch.empty(t, H, dtype=self.dtype, device=self.device)
                ops.row_rmsnorm(x, L.ln2, eps, t, ws=self.ws, splits=so, residual=residual)
            else:
                x = y
                self.comm.all_reduce(x)
                ops.fused_add_rmsnorm(x, residual, L.ln2, eps)
            sg, h = self._lin(x, L, "gu")
            if sg:  # split-K gate_up slabs -> SiLU-mul reduces them
                h = torch.empty(t, cfg.intermediate_size // self.tp, dtype=self.dtype,
                                device=self.device)
                ops.slab_silu(self.ws, sg, t, h.shape[1], h, interleaved=self.gu_il)
            slab, y = self._lin(h, L, "down")
            if tps:
                pend, slab = (slab, y), 0
            elif not slab:
                x = y
                self.comm.all_reduce(x)
        if pend is not None:   # the last layer's down partial: all-reduce, then the final norm
            if pend[0]:
                x = torch.empty(t, H, dtype=self.dtype, device=self.device)
                ops.slab_store(self.ws, pend[0], t, H, x)
            else:
                x = pend[1]
            self.comm.all_reduce(x)
        elif slab:
            x = torch.empty(t, H, dtype=self.dtype, device=self.device)
            ops.slab_store(self.ws, slab, t, H, x)
        idx = meta.logits_indices
        if idx.numel() != t:
            x = x.index_select(0, idx)
            residual = residual.index_select(0, idx)
        else:
            residual = residual.clone()
        ops.fused_add_rmsnorm(x, residual, self.norm, eps)
        return x

    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        """[B, H] -> [B, V] logits (bf16 on GPU; vocab-parallel shards gathered)."""
        if self.lm_head_pk is not None:
            logits = self._packed(h, self.lm_head_pk, "lm")[1]
        else:
            logits = F.linear(h, self.lm_head)
        return self.comm.all_gather_last(logits)
