"""Batch-invariant mode (ENGINE_BATCH_INVARIANT): a sequence's numerics do not depend
on what else shares its steps.  Kernel level: the xr decode GEMM and packed_gemm
give the same bits per row at the INV_PLAN splits; the fixed-piece decode attention
gives a sequence the same bits alone or in any batch; the per-row-rescale prefill
attention with a fixed-chunk plan gives a token the same bits however its prompt is
chunked or batched.  Engine level: greedy tokens of a prompt alone == with other
prompts arriving around it.  (vLLM's VLLM_BATCH_INVARIANT is the reference
behaviour; /root/reference itself serves through vLLM / Ollama,
/root/reference/docker-compose.vllm.yml:42.)"""
import numpy as np
import pytest
import torch

from fasttalk_llm_microservice_amd import ops
from fasttalk_llm_microservice_amd.models import llama
from fasttalk_llm_microservice_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("proj,n,k", [("qkv", 3072, 2048), ("o", 2048, 2048), ("gu", 8192, 2048),
                                      ("down", 2048, 4096), ("lm", 32000, 2048)])
def test_invariant_gemm_rows_match_bitwise(proj, n, k):
    """INV_PLAN (nt, splits): xr at <= 64 rows and packed_gemm at any larger row count
    (every tile config) leave identical slabs / outputs for the shared rows."""
    torch.manual_seed(0)
    nt, sp = llama.INV_PLAN[proj]
    kc = 512 if nt == 2 else 256
    while sp > 1 and k % (kc * sp):
        sp //= 2
    wp = ops.pack_weight((torch.randn(n, k, device=DEV) * 0.05).bfloat16())
    x = torch.randn(300, k, device=DEV).bfloat16()
    gu = proj == "gu"
    u = -6 if gu else -5

    def run_xr(rows):
        ws = torch.full((max(1, sp) * rows * n,), float("nan"), device=DEV)
        if sp > 1:
            ops.skinny_gemm(x[:rows], wp, ws=ws, splits=sp, nt=nt, u=u)
            return ws.view(sp, rows, n)
        return ops.skinny_gemm(x[:rows], wp, splits=1, nt=nt, u=u)

    def run_pg(rows, cfg):
        ws = torch.full((max(1, sp) * rows * n,), float("nan"), device=DEV)
        if sp > 1:
            ops.packed_gemm(x[:rows], wp, ws=ws, splits=sp, epi="slab", cfg=cfg)
            return ws.view(sp, rows, n)
        return ops.packed_gemm(x[:rows], wp, epi="silu" if gu else "store", cfg=cfg)

    def rows_of(y, r):
        return y[:, :r] if sp > 1 else y[:r]

    base = run_xr(50)
    assert torch.isfinite(base.float()).all()
    for rows in (17, 64):
        assert torch.equal(rows_of(run_xr(rows), 17), rows_of(base, 17)), f"xr {rows} rows"
    for rows, cfg in ((300, 0), (300, 5), (130, 1), (200, 2), (260, 6), (256, 3)):
        assert torch.equal(rows_of(run_pg(rows, cfg), 50), base), f"packed_gemm cfg {cfg} at {rows}"


def _decode_batch(lens, bt_rows, k, v, q_rows, piece, nq=32, nkv=8, d=128):
    b = len(lens)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    bt = torch.stack(bt_rows).to(DEV)
    q = torch.stack(q_rows)
    n_out, n_ml = ops.decode_workspace(b, nq, nkv, d, piece=piece, max_len=bt.shape[1] * 16)
    tmp_out = torch.full((n_out,), float("nan"), device=DEV)
    tmp_ml = torch.full((n_ml,), float("nan"), device=DEV)
    cnt = ops.decode_counters(b, nkv, DEV)
    out = torch.full((b, nq * d), float("nan"), device=DEV).bfloat16()
    ops.decode_attention(out, q, k, v, bt, sl, tmp_out, tmp_ml, nq, nkv, d, d ** -0.5,
                         counters=cnt, piece=piece)
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0, "combine tickets must be left zeroed"
    return out, sl, bt, q


@pytest.mark.parametrize("target_len", [100, 513, 3000, 8192])
def test_decode_attention_piece_mode_is_batch_invariant(target_len):
    """A sequence's output row is bit-identical alone and inside batches of other
    lengths (the flattened partition moves its split points with the batch; pieces
    do not), and matches the fp32 reference."""
    torch.manual_seed(target_len)
    nq, nkv, d, bs = 32, 8, 128, 16
    maxb = 8192 // bs
    nblocks = 64 * maxb // 4
    k = torch.randn(nblocks, nkv, bs, d, device=DEV).bfloat16()
    v = torch.randn(nblocks, nkv, d, bs, device=DEV).bfloat16()
    g = torch.Generator().manual_seed(1)

    def row(length):
        r = torch.zeros(maxb, dtype=torch.int32)
        nb = -(-length // bs)
        r[:nb] = torch.randint(0, nblocks, (nb,), generator=g, dtype=torch.int32)
        return r

    t_bt = row(target_len)
    t_q = torch.randn(nq * d, device=DEV).bfloat16()
    alone, sl, bt, q = _decode_batch([target_len], [t_bt], k, v, [t_q], ops.DECODE_INV_PIECE)
    expect = ref.paged_attention(q.view(1, nq, d), k, v, bt, sl, torch.arange(2, dtype=torch.int32),
                                 d ** -0.5).view(1, nq * d)
    a = alone.float().cpu()
    e = expect.float().cpu()
    assert ((a - e).abs() <= 2e-2 + 2e-2 * e.abs()).all()
    for others, pos in (([7, 3000, 250], 1), ([4000] * 40 + [17] * 9, 33), ([1] * 63, 63)):
        lens = list(others)
        lens.insert(pos, target_len)
        bts = [row(x) for x in others]
        bts.insert(pos, t_bt)
        qs = [torch.randn(nq * d, device=DEV).bfloat16() for _ in others]
        qs.insert(pos, t_q)
        out, *_ = _decode_batch(lens, bts, k, v, qs, ops.DECODE_INV_PIECE)
        assert torch.equal(out[pos], alone[0]), f"batch of {len(lens)}"


def _prefill_call(chunks, k, v, bt_rows, q_all, nq, nkv, d, invariant=True):
    """chunks: [(seq index into bt_rows / q_all, first new token s, new tokens n, the
    sequence's cached prefix c)]: new token j sits at position c + j -> {(seq, j): row}."""
    lens = [c + s + n for _, s, n, c in chunks]
    qlens = [n for _, _, n, _ in chunks]
    qsl = torch.tensor([0] + list(np.cumsum(qlens)), dtype=torch.int32)
    t = int(qsl[-1])
    q = torch.cat([q_all[i][s:s + n] for i, s, n, _ in chunks])
    bt = torch.stack([bt_rows[i] for i, *_ in chunks]).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    tiles, comb = ops.build_prefill_tiles(qlens, ops.prefill_tile_tokens(nq, nkv), seq_lens=lens,
                                          nkv=nkv, fixed_chunk=ops.PREFILL_INV_CHUNK if invariant else 0,
                                          max_partials=512)
    ti = torch.tensor(tiles, dtype=torch.int32, device=DEV).flatten()
    out = torch.full((t, nq * d), float("nan"), device=DEV).bfloat16()
    n_po, n_pml = ops.prefill_partials(nkv, d, 512)
    po = torch.full((n_po,), float("nan"), device=DEV)
    pml = torch.full((n_pml,), float("nan"), device=DEV)
    cb = torch.tensor(comb or [[0, 0, 0, 0]], dtype=torch.int32, device=DEV).flatten()
    ops.prefill_attention(out, q, k, v, bt, sl, qsl.to(DEV), ti, len(tiles), nq, nkv, d, d ** -0.5,
                          po, pml, cb, len(comb), sum(c[3] for c in comb), invariant=invariant)
    res = {}
    for j, (i, s, n, _) in enumerate(chunks):
        for tok in range(n):
            res[(i, s + tok)] = out[int(qsl[j]) + tok]
    return res


def test_prefill_attention_invariant_to_chunking_and_batch():
    """Every prompt token's attention output is bit-identical whether its prompt is
    prefilled in one chunk, in chunks cut elsewhere, or batched with other prompts
    (cached prefixes of 0, 1.5k and 2.9k tokens), and matches the reference."""
    torch.manual_seed(3)
    nq, nkv, d, bs = 32, 8, 128, 16
    maxb = 4096 // bs
    nblocks = 3 * maxb
    k = torch.randn(nblocks, nkv, bs, d, device=DEV).bfloat16()
    v = torch.randn(nblocks, nkv, d, bs, device=DEV).bfloat16()
    perm = torch.randperm(nblocks).int()
    bt_rows = [perm[i * maxb:(i + 1) * maxb] for i in range(3)]
    newt = [150, 300, 200]   # new tokens over cached prefixes of 2900, 1500 and 0
    q_all = [torch.randn(n, nq * d, device=DEV).bfloat16() for n in newt]
    one = _prefill_call([(0, 0, 150, 2900)], k, v, bt_rows, q_all, nq, nkv, d)
    two = _prefill_call([(0, 0, 70, 2900)], k, v, bt_rows, q_all, nq, nkv, d)
    two.update(_prefill_call([(0, 70, 80, 2900)], k, v, bt_rows, q_all, nq, nkv, d))
    batched = _prefill_call([(1, 0, 300, 1500), (0, 0, 33, 2900), (2, 0, 200, 0)], k, v, bt_rows,
                            q_all, nq, nkv, d)
    batched.update(_prefill_call([(2, 0, 5, 0), (0, 33, 117, 2900)], k, v, bt_rows, q_all, nq, nkv, d))
    for tok in range(150):
        assert torch.equal(one[(0, tok)], two[(0, tok)]), f"token {tok}: one vs two chunks"
        assert torch.equal(one[(0, tok)], batched[(0, tok)]), f"token {tok}: alone vs batched"
    # correctness of the invariant kernel against the fp32 reference
    L = torch.tensor([3050], dtype=torch.int32, device=DEV)
    qsl = torch.tensor([0, 150], dtype=torch.int32)
    expect = ref.paged_attention(q_all[0].view(150, nq, d), k, v, bt_rows[0][None].to(DEV), L, qsl,
                                 d ** -0.5).view(150, nq * d).float().cpu()
    got = torch.stack([one[(0, t)] for t in range(150)]).float().cpu()
    assert ((got - expect).abs() <= 2e-2 + 2e-2 * expect.abs()).all()


def _target_logits(batch_invariant: bool):
    """(alone, mixed) per-step logits rows of one greedy prompt: decoded alone, then
    with other prompts of other lengths arriving around it."""
    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    eng = LLMEngine(EngineConfig(model="tiny-2k", device="cuda", num_kv_blocks=1024,
                                 max_model_len=4096, max_num_seqs=16,
                                 batch_invariant=batch_invariant, enable_prefix_caching=False))
    assert eng.runner.model.invariant == batch_invariant
    rng = np.random.default_rng(5)
    target = rng.integers(0, 120000, 1300).tolist()
    others = [rng.integers(0, 120000, n).tolist() for n in (40, 700, 2100, 9, 333)]
    r = eng.runner

    def run(schedule):
        toks = []
        step = 0
        r.logits_tap, r.logits_tap_ids = [], []
        eng.add_request("t", target, SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True))
        while eng.has_work() or schedule:
            while schedule and schedule[0][0] <= step:
                _, i = schedule.pop(0)
                eng.add_request(f"o{i}-{step}", others[i],
                                SamplingParams(temperature=0.0, max_tokens=30, ignore_eos=True))
            for o in eng.step():
                if o.request_id == "t":
                    toks.extend(o.token_ids)
            step += 1
        torch.cuda.synchronize()
        logits = [lg[row].float().cpu() for lg, ids in zip(r.logits_tap, r.logits_tap_ids)
                  for row, rid in enumerate(ids or []) if rid == "t"]
        shared = max(len(ids) for ids in r.logits_tap_ids if ids and "t" in ids)
        r.logits_tap = r.logits_tap_ids = None
        return toks, logits, shared

    alone = run([])
    mixed = run([(0, 0), (0, 1), (2, 2), (5, 3), (9, 4), (20, 1)])
    return alone, mixed


def test_engine_batch_invariant_logits():
    """Batch-invariant engine: every step's logits row of the target is bit-identical
    alone and while 6 other prompts share its steps (mixed prefill steps, decode
    batches of changing size), so its greedy tokens are too."""
    (ta, la, n1), (tm, lm, n2) = _target_logits(True)
    # (a pipelined run may tap one queued step past the last token: >= 40 rows)
    assert len(ta) == 40 and len(la) >= 40 and len(lm) >= 40 and n1 == 1
    assert n2 >= 4, n2   # the target really shared its steps
    assert tm == ta
    for k, (a, b) in enumerate(zip(la[:40], lm[:40])):
        assert torch.equal(a, b), f"step {k}"


def test_engine_default_mode_is_not_batch_invariant():
    """Control for the test above: the default plans (fused decode layer for small
    batches, packed_gemm rows in mixed steps, batch-dependent attention splits)
    change the target's logits bits when others share its steps."""
    (_, la, _), (_, lm, n2) = _target_logits(False)
    assert n2 >= 4
    assert any(not torch.equal(a, b) for a, b in zip(la, lm))
