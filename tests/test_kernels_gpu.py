"""Numerics of every gfx950 HIP kernel against the fp32 PyTorch reference of the
same op (fasttalk_llm_microservice_amd/ops/reference.py)."""
import math

import pytest
import torch

from fasttalk_llm_microservice_amd import ops
from fasttalk_llm_microservice_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=0.0, msg=""):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{msg}: {bad} elems out of tol, max err {err.max().item():.4g}"


@pytest.fixture(autouse=True)
def _native_loaded():
    ops.native()  # fail loudly if the extension is missing
    torch.manual_seed(0)


@pytest.mark.parametrize("hidden", [2048, 3072, 4096, 8192])
@pytest.mark.parametrize("rows", [1, 7, 130])
def test_rmsnorm(hidden, rows):
    x = torch.randn(rows, hidden, device=DEV).bfloat16()
    w = (1 + 0.1 * torch.randn(hidden, device=DEV)).bfloat16()
    out = ops.rmsnorm(x, w, 1e-5)
    _close(out, ref.rmsnorm(x, w, 1e-5), atol=2e-2, rtol=1e-2, msg="rmsnorm")


@pytest.mark.parametrize("hidden", [2048, 4096])
def test_fused_add_rmsnorm(hidden):
    x = torch.randn(33, hidden, device=DEV).bfloat16()
    r = torch.randn(33, hidden, device=DEV).bfloat16()
    w = (1 + 0.1 * torch.randn(hidden, device=DEV)).bfloat16()
    ey, er = ref.fused_add_rmsnorm(x, r, w, 1e-5)
    ops.fused_add_rmsnorm(x, r, w, 1e-5)
    _close(r, er, atol=1e-2, rtol=1e-2, msg="residual")
    _close(x, ey, atol=2e-2, rtol=1e-2, msg="normed")


def test_silu_mul():
    gu = torch.randn(37, 2 * 14336, device=DEV).bfloat16()
    _close(ops.silu_mul(gu), ref.silu_mul(gu), atol=2e-2, rtol=1e-2, msg="silu_mul")


def _alloc_cache(nblocks, nkv, bs, d):
    """K blocks [nkv, bs, d]; V blocks transposed [nkv, d, bs] (the engine's layout)."""
    k = torch.randn(nblocks, nkv, bs, d, device=DEV).bfloat16()
    v = torch.randn(nblocks, nkv, d, bs, device=DEV).bfloat16()
    return k, v


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (24, 8, 128), (32, 8, 64), (8, 1, 128)])
def test_rope_kv_write(nq, nkv, d):
    t, bs, nblocks = 45, 16, 20
    qkv = torch.randn(t, (nq + 2 * nkv) * d, device=DEV).bfloat16()
    pos = torch.randint(0, 4000, (t,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(d, 8192, 500000.0, {"factor": 8.0, "low_freq_factor": 1.0,
                                              "high_freq_factor": 4.0,
                                              "original_max_position_embeddings": 8192}, DEV)
    slots = torch.randperm(nblocks * bs, device=DEV)[:t].int()
    slots[3] = -1
    k1, v1 = _alloc_cache(nblocks, nkv, bs, d)
    k2, v2 = k1.clone(), v1.clone()
    q1 = qkv.clone()
    q2 = qkv.clone()
    ops.rope_kv_write(q1, pos, cs, slots, k1, v1, nq, nkv, d)
    ref.rope_kv_write(q2, pos, cs, slots, k2, v2, nq, nkv, d)
    _close(q1[:, : nq * d], q2[:, : nq * d], atol=2e-2, rtol=1e-2, msg="q")
    _close(k1, k2, atol=2e-2, rtol=1e-2, msg="k cache")
    assert torch.equal(v1, v2)


def _random_tables(lens, bs, nblocks_total):
    perm = torch.randperm(nblocks_total).int()
    maxb = max((l + bs - 1) // bs for l in lens)
    bt = torch.zeros(len(lens), maxb, dtype=torch.int32)
    i = 0
    for b, l in enumerate(lens):
        n = (l + bs - 1) // bs
        bt[b, :n] = perm[i: i + n]
        i += n
    return bt


def _decode_case(lens, nq, nkv, d, bs=16, seed=0, fused=True, calls=1):
    torch.manual_seed(seed)
    nblocks = sum((l + bs - 1) // bs for l in lens) + 4
    k, v = _alloc_cache(nblocks, nkv, bs, d)
    bt = _random_tables(lens, bs, nblocks).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    b = len(lens)
    q = torch.randn(b, nq * d, device=DEV).bfloat16()
    n_out, n_ml = ops.decode_workspace(b, nq, nkv, d)
    tmp_out = torch.full((n_out,), float("nan"), device=DEV)
    tmp_ml = torch.full((n_ml,), float("nan"), device=DEV)
    out = torch.full((b, nq * d), float("nan"), device=DEV).bfloat16()
    scale = d ** -0.5
    cnt = ops.decode_counters(b, nkv, DEV) if fused else None
    for _ in range(calls):
        first = out.clone()
        ops.decode_attention(out, q, k, v, bt, sl, tmp_out, tmp_ml, nq, nkv, d, scale, counters=cnt)
    if calls > 1:   # the in-launch combine's tickets reset: repeat calls agree bit for bit
        assert torch.equal(first, out)
    if cnt is not None:
        torch.cuda.synchronize()
        assert int(cnt.abs().sum()) == 0, "combine tickets must be left zeroed"
    expect = ref.paged_attention(q.view(b, nq, d), k, v, bt, sl,
                                 torch.arange(b + 1, dtype=torch.int32), scale).view(b, nq * d)
    return out, expect


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (64, 8, 128), (8, 8, 128), (24, 8, 128),
                                      (32, 8, 64), (8, 1, 128), (16, 8, 128)])
@pytest.mark.parametrize("fused", [True, False])
def test_decode_attention(nq, nkv, d, fused):
    # lengths around tile / block edges; one long sequence spreads over many waves;
    # fused = segments shared by several waves merged inside the launch (tickets)
    out, expect = _decode_case([1, 17, 255, 256, 257, 1000, 2100], nq, nkv, d, fused=fused,
                               calls=3)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="decode attention")


@pytest.mark.parametrize("b,max_len", [(1, 8192), (50, 6000), (64, 8192), (256, 700)])
def test_decode_attention_serving_shapes(b, max_len):
    """Headline shapes: ragged contexts up to max_model_len at the 50/64-row buckets."""
    g = torch.Generator().manual_seed(b)
    lens = torch.randint(max(1, max_len // 4), max_len + 1, (b,), generator=g).tolist()
    lens[0] = max_len
    out, expect = _decode_case(lens, 32, 8, 128, seed=b, calls=2)
    assert torch.isfinite(out.float()).all()
    _close(out, expect, atol=2e-2, rtol=2e-2, msg=f"decode attention b={b}")


@pytest.mark.parametrize("bs", [32, 64])
def test_decode_attention_block_sizes(bs):
    out, expect = _decode_case([5, 64, 300, 1025], 32, 8, 128, bs=bs)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg=f"decode attention bs={bs}")


def _prefill_run(seqs, nq, nkv, d, split, num_cus=256, seed=0):
    """(out, expect) of the prefill kernel over (new tokens, cached prefix) pairs;
    split: plan split-KV items (partials + combine) with this many CUs."""
    torch.manual_seed(seed)
    bs = 16
    lens = [a + p for a, p in seqs]
    nblocks = sum((l + bs - 1) // bs for l in lens) + 4
    k, v = _alloc_cache(nblocks, nkv, bs, d)
    bt = _random_tables(lens, bs, nblocks).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    qlens = [a for a, _ in seqs]
    qsl = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32)
    t = int(qsl[-1])
    q = torch.randn(t, nq * d, device=DEV).bfloat16()
    tiles, comb = ops.build_prefill_tiles(qlens, ops.prefill_tile_tokens(nq, nkv),
                                          seq_lens=lens if split else None, nkv=nkv, num_cus=num_cus,
                                          min_split_tiles=1)
    assert bool(comb) == bool(split), comb
    ti = torch.tensor(tiles, dtype=torch.int32, device=DEV).flatten()
    out = torch.zeros(t, nq * d, device=DEV).bfloat16()
    scale = d ** -0.5
    if comb:
        n_po, n_pml = ops.prefill_partials(nkv, d)
        po = torch.full((n_po,), float("nan"), device=DEV)
        pml = torch.full((n_pml,), float("nan"), device=DEV)
        cb = torch.tensor(comb, dtype=torch.int32, device=DEV).flatten()
        ops.prefill_attention(out, q, k, v, bt, sl, qsl.to(DEV), ti, len(tiles), nq, nkv, d, scale,
                              po, pml, cb, len(comb), sum(c[3] for c in comb))
    else:
        ops.prefill_attention(out, q, k, v, bt, sl, qsl.to(DEV), ti, len(tiles), nq, nkv, d, scale)
    expect = ref.paged_attention(q.view(t, nq, d), k, v, bt, sl, qsl, scale).view(t, nq * d)
    return out, expect


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (24, 8, 128), (64, 8, 128), (32, 8, 64),
                                      (8, 8, 128)])
def test_prefill_attention(nq, nkv, d):
    # (new tokens, cached prefix)
    seqs = [(1, 0), (5, 0), (64, 0), (77, 33), (16, 300), (130, 1), (3, 500)]
    out, expect = _prefill_run(seqs, nq, nkv, d, split=False)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="prefill attention")


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (32, 8, 64), (8, 8, 128)])
def test_prefill_attention_split_kv(nq, nkv, d):
    """Split-KV work items (history ranges over several workgroups, fp32 partials
    merged by the combine kernel): chat-turn shapes (~100 new tokens over long
    cached histories), ranges cut at arbitrary tiles incl. ones entirely above a
    query block's early rows (fully masked partials)."""
    seqs = [(100, 2900), (37, 4000), (64, 0), (130, 700), (3, 1500), (1, 63)]
    out, expect = _prefill_run(seqs, nq, nkv, d, split=True, num_cus=256)
    assert torch.isfinite(out.float()).all()
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="prefill attention split-KV")


def test_prefill_attention_strided_q():
    """q read straight out of the fused QKV buffer (row stride > nq*d)."""
    nq, nkv, d, bs = 32, 8, 128, 16
    lens = [40, 90]
    nblocks = 16
    k, v = _alloc_cache(nblocks, nkv, bs, d)
    bt = _random_tables(lens, bs, nblocks).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    qsl = torch.tensor([0, 40, 130], dtype=torch.int32)
    qkv = torch.randn(130, (nq + 2 * nkv) * d, device=DEV).bfloat16()
    tiles, _ = ops.build_prefill_tiles([40, 90], ops.prefill_tile_tokens(nq, nkv))
    ti = torch.tensor(tiles, dtype=torch.int32, device=DEV).flatten()
    out = torch.zeros(130, nq * d, device=DEV).bfloat16()
    ops.prefill_attention(out, qkv, k, v, bt, sl, qsl.to(DEV), ti, len(tiles), nq, nkv, d, 0.088)
    expect = ref.paged_attention(qkv[:, : nq * d].reshape(130, nq, d), k, v, bt, sl, qsl,
                                 0.088).view(130, nq * d)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="strided q")


def _sp(b, temp, top_p=1.0, top_k=0):
    return (torch.full((b,), temp, device=DEV), torch.full((b,), top_p, device=DEV),
            torch.full((b,), top_k, dtype=torch.int32, device=DEV),
            torch.arange(b, dtype=torch.int64, device=DEV) * 7919,
            torch.zeros(b, dtype=torch.int32, device=DEV))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sample_greedy(dtype):
    logits = torch.randn(50, 128256, device=DEV).to(dtype)
    t, p, k, s, st = _sp(50, 0.0)
    out = ops.sample(logits, t, p, k, s, st)
    assert torch.equal(out.long().cpu(), logits.float().argmax(-1).cpu())


def test_sample_topk1_is_argmax():
    # bf16 logits (the engine's dtype): the draw must hit a maximal logit (ties
    # at bf16 resolution are legitimately interchangeable)
    logits = torch.randn(20, 128256, device=DEV).bfloat16()
    t, p, k, s, st = _sp(20, 0.8, 1.0, 1)
    out = ops.sample(logits, t, p, k, s, st).long().cpu()
    lf = logits.float().cpu()
    assert all(lf[i, out[i]] == lf[i].max() for i in range(20))


def test_sample_topk_membership():
    logits = torch.randn(64, 128256, device=DEV).bfloat16()
    t, p, k, s, st = _sp(64, 1.0, 1.0, 40)
    out = ops.sample(logits, t, p, k, s, st).long().cpu()
    lf = logits.float().cpu()
    kth = lf.topk(40, dim=-1).values[:, -1]
    assert all(lf[i, out[i]].item() >= kth[i].item() for i in range(64))


@pytest.mark.parametrize("kk", [3, 40, 64, 100])
def test_sample_topk_exact_set(kk):
    """At a huge temperature the kept set is drawn ~uniformly: over many seeds
    every one of the k largest logits (distinct values) must show up and no other
    id, so the top-k threshold search is exact, not just conservative."""
    b, v = 512, 128256
    base = torch.randn(v) * 0.5
    top = torch.randperm(v)[:kk]
    base[top] = 4.0 + 0.0625 * torch.arange(kk, dtype=torch.float32)  # exact in bf16
    logits = base.to(DEV).bfloat16().unsqueeze(0).repeat(b, 1)
    t, p, k, s, st = _sp(b, 1e4, 1.0, kk)
    out = set(ops.sample(logits, t, p, k, s, st).long().cpu().tolist())
    assert out == set(top.tolist())


@pytest.mark.parametrize("top_p", [1.0, 0.6])
def test_sample_topk_distribution(top_p):
    """Multi-workgroup top-k path (k <= 64): draws follow softmax over the k largest
    logits (then the top-p nucleus of those), the kept ids spread over several
    vocabulary slices; repeat calls with the same (seed, step) are identical."""
    v, rows, kk = 128256, 2048, 5
    base = torch.full((v,), -3.0)
    top = torch.tensor([7, 20000, 64001, 90000, 128000, 5000])   # 6 ids in 5 slices
    base[top] = torch.tensor([2.0, 1.5, 1.25, 1.0, 0.5, 0.25])
    logits = base.to(DEV).bfloat16().unsqueeze(0).repeat(rows, 1)
    t = torch.full((rows,), 0.8, device=DEV)
    p = torch.full((rows,), top_p, device=DEV)
    k = torch.full((rows,), kk, dtype=torch.int32, device=DEV)
    s = torch.arange(rows, dtype=torch.int64, device=DEV) * 7919 + 11
    counts = torch.zeros(v)
    for step in range(4):
        st = torch.full((rows,), step, dtype=torch.int32, device=DEV)
        out = ops.sample(logits, t, p, k, s, st)
        assert torch.equal(out, ops.sample(logits, t, p, k, s, st))
        counts += torch.bincount(out.long().cpu(), minlength=v).float()
    kept = top[:kk]
    pr = torch.softmax(base[kept].bfloat16().float() / 0.8, -1)
    above = torch.cumsum(pr, 0) - pr
    member = above < top_p if top_p < 1 else torch.ones(kk, dtype=torch.bool)
    expect = torch.zeros(v)
    expect[kept[member]] = pr[member] / pr[member].sum()
    emp = counts / counts.sum()
    assert counts[expect == 0].sum() == 0
    assert (emp - expect).abs().max().item() < 0.015


def test_sample_topk_ties_fall_back():
    """More tied candidates than a slice holds (flat logits): the row is finished by
    the one-workgroup kernel, still inside the tie set."""
    v = 128256
    logits = torch.zeros(4, v, device=DEV).bfloat16()
    logits[:, 1000:1300] = 1.0          # 300 tied maxima in one slice
    t, p, k, s, st = _sp(4, 1.0, 1.0, 40)
    out = ops.sample(logits, t, p, k, s, st).long().cpu()
    assert all(1000 <= int(o) < 1300 for o in out)


def test_sample_topp_membership():
    logits = torch.randn(64, 32000, device=DEV) * 4
    t, p, k, s, st = _sp(64, 0.7, 0.5, 0)
    out = ops.sample(logits, t, p, k, s, st).long().cpu()
    probs = torch.softmax(logits.cpu() / 0.7, -1)
    for i in range(64):
        sp, si = probs[i].sort(descending=True)
        n = int((sp.cumsum(0) < 0.5).sum().item()) + 1
        assert out[i].item() in set(si[: n + 1].tolist())


def test_sample_distribution():
    """Empirical frequencies of many independent draws match softmax(logits/T)."""
    v = 64
    base = torch.randn(v) * 1.5
    rows = 4096
    logits = base.to(DEV).repeat(rows, 1)
    t = torch.full((rows,), 0.9, device=DEV)
    p = torch.ones(rows, device=DEV)
    k = torch.zeros(rows, dtype=torch.int32, device=DEV)
    s = torch.arange(rows, dtype=torch.int64, device=DEV) * 104729 + 17
    counts = torch.zeros(v)
    for step in range(8):
        st = torch.full((rows,), step, dtype=torch.int32, device=DEV)
        out = ops.sample(logits, t, p, k, s, st).long().cpu()
        counts += torch.bincount(out, minlength=v).float()
    emp = counts / counts.sum()
    expect = torch.softmax(base / 0.9, -1)
    assert (emp - expect).abs().max().item() < 0.01


def test_sample_topp_distribution_is_exact():
    """top_p = 0.3 on a flat-tailed distribution: acceptance per rejection round is
    only ~0.3, so ~6% of rows exhaust the 8 rounds and take the exact nucleus
    fallback -- the draws must still follow the renormalised nucleus (ADVICE r1:
    the old argmax fallback biased them towards greedy)."""
    v = 64
    base = torch.linspace(2.0, -2.0, v)   # distinct logits (no ties at the nucleus edge)
    rows = 4096
    logits = base.to(DEV).repeat(rows, 1)
    t = torch.ones(rows, device=DEV)
    p = torch.full((rows,), 0.3, device=DEV)
    k = torch.zeros(rows, dtype=torch.int32, device=DEV)
    s = torch.arange(rows, dtype=torch.int64, device=DEV) * 7919 + 3
    counts = torch.zeros(v)
    for step in range(8):
        st = torch.full((rows,), step, dtype=torch.int32, device=DEV)
        out = ops.sample(logits, t, p, k, s, st).long().cpu()
        counts += torch.bincount(out, minlength=v).float()
    probs = torch.softmax(base, -1)
    order = probs.argsort(descending=True)
    above = torch.cumsum(probs[order], 0) - probs[order]     # strictly more likely mass
    nucleus = order[above < 0.3]
    expect = torch.zeros(v)
    expect[nucleus] = probs[nucleus] / probs[nucleus].sum()
    emp = counts / counts.sum()
    assert counts[[i for i in range(v) if i not in set(nucleus.tolist())]].sum() == 0
    assert (emp - expect).abs().max().item() < 0.012, (emp[nucleus], expect[nucleus])


def test_sample_mask():
    v = 1000
    logits = torch.randn(8, v, device=DEV)
    mask = torch.zeros(8, (v + 31) // 32, dtype=torch.int32)
    allowed = [5, 77, 999]
    for a in allowed:
        mask[:, a // 32] |= (1 << (a % 32)) if a % 32 < 31 else -(1 << 31)
    t, p, k, s, st = _sp(8, 1.0)
    out = ops.sample(logits, t, p, k, s, st, mask=mask.to(DEV)).cpu().tolist()
    assert all(o in allowed for o in out)
    t0, *_ = _sp(8, 0.0)
    out = ops.sample(logits, t0, p, k, s, st, mask=mask.to(DEV)).cpu()
    exp = torch.tensor(allowed)[logits.cpu()[:, allowed].argmax(-1)]
    assert torch.equal(out.long(), exp)


def test_sample_deterministic():
    logits = torch.randn(16, 128256, device=DEV)
    t, p, k, s, st = _sp(16, 0.7, 0.9, 0)
    a = ops.sample(logits, t, p, k, s, st).cpu()
    b = ops.sample(logits, t, p, k, s, st).cpu()
    assert torch.equal(a, b)


def test_kv_block_copy():
    k, v = _alloc_cache(10, 8, 16, 128)
    k0, v0 = k.clone(), v.clone()
    pairs = torch.tensor([[1, 5], [2, 7]], dtype=torch.int32, device=DEV)
    ops.kv_block_copy(k, v, pairs)
    assert torch.equal(k[5], k0[1]) and torch.equal(v[7], v0[2]) and torch.equal(k[0], k0[0])


def test_kv_swap_gather_scatter():
    layers = [_alloc_cache(12, 8, 16, 128) for _ in range(3)]
    ptrs = torch.tensor([c.data_ptr() for kv in layers for c in kv], dtype=torch.int64, device=DEV)
    be = 8 * 16 * 128
    ids = torch.tensor([7, 0, 11, 3], dtype=torch.int32, device=DEV)
    st = torch.empty(4, 6 * be, dtype=torch.bfloat16, device=DEV)
    ops.kv_swap(layers, ptrs, ids, st, to_staging=True)
    expect = torch.stack([torch.cat([c[b].flatten() for kv in layers for c in kv])
                          for b in ids.tolist()])
    assert torch.equal(st, expect)
    # scatter a new payload into other blocks; untouched blocks stay as they were
    before = [c.clone() for kv in layers for c in kv]
    new = torch.randn(2, 6 * be, device=DEV).bfloat16()
    ids2 = torch.tensor([5, 9], dtype=torch.int32, device=DEV)
    ops.kv_swap(layers, ptrs, ids2, new, to_staging=False)
    flat = [c for kv in layers for c in kv]
    for ci, c in enumerate(flat):
        for i, b in enumerate((5, 9)):
            assert torch.equal(c[b].flatten(), new[i, ci * be:(ci + 1) * be])
        keep = [b for b in range(12) if b not in (5, 9)]
        assert torch.equal(c[keep], before[ci][keep])


# ----------------------------------------------------------------------------------
# W4A16 (AWQ-style int4, group 128)
# ----------------------------------------------------------------------------------

def _w4(n, k, seed=0):
    from fasttalk_llm_microservice_amd.ops import quant as Q

    g = torch.Generator().manual_seed(seed)
    w = torch.randn(n, k, generator=g) * 0.05
    q, z, s = Q.quantize_w4(w)
    return Q, Q.pack_w4(q.to(DEV), z.to(DEV), s.to(DEV)), Q.dequantize_w4(q, z, s)


@pytest.mark.parametrize("n,k", [(1024, 4096), (512, 1024), (4096, 14336), (6144, 4096)])
def test_w4_dequant_exact(n, k):
    Q, W, ref_w = _w4(n, k)
    out = Q.w4_dequant(W)
    assert torch.equal(out.float().cpu(), ref_w.bfloat16().float())


@pytest.mark.parametrize("m", [1, 5, 16, 29, 48, 64])
@pytest.mark.parametrize("n,k,nt,splits", [(1024, 4096, 1, 1), (1024, 4096, 2, 1),
                                           (2048, 4096, 4, 1), (512, 1024, 1, 2),
                                           (4096, 14336, 1, 4), (1024, 4096, 2, 2)])
def test_w4_gemm_matches_fp32(m, n, k, nt, splits):
    Q, W, ref_w = _w4(n, k, seed=m)
    x = torch.randn(m, k, generator=torch.Generator().manual_seed(7)).bfloat16()
    ref_y = x.float() @ ref_w.t()
    xd = x.to(DEV)
    if splits == 1:
        y = Q.w4_gemm(xd, W, nt=nt).float().cpu()
        tol = 2e-2 * ref_y.abs().max().item() + 1e-2
        assert (y - ref_y).abs().max().item() < tol
    ws = torch.full((splits * m * n,), float("nan"), device=DEV)
    Q.w4_gemm(xd, W, ws=ws, splits=splits, nt=nt)
    y = ws.view(splits, m, n).sum(0).cpu()
    assert (y - ref_y).abs().max().item() < 1e-3 * ref_y.abs().max().item() + 1e-3


@pytest.mark.parametrize("xr", [1, 4, 5])
@pytest.mark.parametrize("m", [17, 33, 50, 64])
@pytest.mark.parametrize("n,k,nt,splits", [(1024, 4096, 1, 1), (2048, 4096, 2, 2), (2048, 4096, 4, 1),
                                           (1024, 14336, 1, 4), (2048, 14336, 2, 7),
                                           (1024, 4096, 1, 4), (1024, 4096, 1, 8)])
def test_w4_xr_gemm_matches_fp32(m, n, k, nt, splits, xr):
    """The x-in-LDS W4A16 variants (17..64 rows; xr 4 / 5 = "mh": two tiles per wave,
    rows over wave pairs, zero-point term by f32 MFMAs after the loop): bf16 out and
    split-K fp32 slabs."""
    from fasttalk_llm_microservice_amd.models.llama import w4_fits

    if not w4_fits(xr, nt, splits, n, k):
        pytest.skip("shape outside this kernel's tiling")
    Q, W, ref_w = _w4(n, k, seed=m + 1)
    x = torch.randn(m, k, generator=torch.Generator().manual_seed(9)).bfloat16()
    ref_y = x.float() @ ref_w.t()
    xd = x.to(DEV)
    if splits == 1:
        y = Q.w4_gemm(xd, W, nt=nt, xr=xr).float().cpu()
        assert (y - ref_y).abs().max().item() < 2e-2 * ref_y.abs().max().item() + 1e-2
    ws = torch.full((splits * m * n,), float("nan"), device=DEV)
    Q.w4_gemm(xd, W, ws=ws, splits=splits, nt=nt, xr=xr)
    y = ws.view(splits, m, n).sum(0).cpu()
    assert (y - ref_y).abs().max().item() < 1e-3 * ref_y.abs().max().item() + 1e-3


@pytest.mark.parametrize("xr", [1, 4, 5])
@pytest.mark.parametrize("m", [20, 50, 64])
def test_w4_xr_silu_epilogue(m, xr):
    """gate_up quantized with its rows interleaved in 16-row groups: the W4 xr
    kernel's SiLU epilogue returns h = silu(gate) * up."""
    from fasttalk_llm_microservice_amd import ops as O
    from fasttalk_llm_microservice_amd.ops import quant as Q

    inter, k = 1024, 4096
    g = torch.Generator().manual_seed(m)
    w = torch.randn(2 * inter, k, generator=g) * 0.05
    wi = O.interleave_gate_up(w, 1)
    q, z, s = Q.quantize_w4(wi)
    W = Q.pack_w4(q.to(DEV), z.to(DEV), s.to(DEV))
    wdq = Q.dequantize_w4(q, z, s)
    x = torch.randn(m, k, generator=torch.Generator().manual_seed(3)).bfloat16()
    y = x.float() @ wdq.t()
    gt, up = y.view(m, -1, 2, 16).unbind(2)
    ref = (torch.nn.functional.silu(gt) * up).reshape(m, inter)
    h = Q.w4_gemm(x.to(DEV), W, nt=2, xr=xr, silu=True).float().cpu()
    assert h.shape == (m, inter)
    assert (h - ref).abs().max().item() < 2e-2 * ref.abs().max().item() + 1e-2


# ----------------------------------------------------------------------------------
# decode-shape skinny GEMM + fused row epilogues
# ----------------------------------------------------------------------------------

@pytest.mark.parametrize("m", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("nt,u,splits", [(1, -3, 1), (2, -3, 4), (4, -3, 2), (1, -4, 1), (2, -4, 2),
                                         (2, -5, 1), (1, -5, 1), (2, -5, 4), (1, -5, 2),
                                         (2, -7, 1), (1, -7, 1), (2, -7, 4), (1, -7, 2)])
def test_skinny_gemm(m, nt, u, splits):
    """Packed-weight decode GEMMs ("pk" u=-3, "xc" u=-4, chunk-pipelined "xr"
    u=-5: 8 / 16 / 2 / 8 chunks per workgroup; u=-7 the same on 8-wave workgroups)
    vs fp32, bf16 out and split-K fp32 slabs."""
    n, k = 1024, 4096
    w = (torch.randn(n, k, device=DEV) * 0.05).bfloat16()
    x = torch.randn(m, k, device=DEV).bfloat16()
    ref_y = x.float() @ w.float().t()
    wp = ops.pack_weight(w)
    if splits == 1:
        y = ops.skinny_gemm(x, wp, nt=nt, u=u).float()
    else:
        ws = torch.empty(splits * m * n, device=DEV)
        ops.skinny_gemm(x, wp, ws=ws, splits=splits, nt=nt, u=u)
        y = ws.view(splits, m, n).sum(0)
    _close(y, ref_y, atol=3e-2, rtol=1e-2, msg="skinny_gemm")


@pytest.mark.parametrize("m", [1, 29, 50, 64])
@pytest.mark.parametrize("n,k", [(2048, 4096), (28672, 4096)])
@pytest.mark.parametrize("u", [-6, -8])
def test_skinny_gemm_xr_silu(m, n, k, u):
    """xr with the SiLU epilogue on an interleave_gate_up(w, 1) image: h = silu(x Wg^T)
    * (x Wu^T) straight from the GEMM (no slabs), vs fp32; u=-8 on 8-wave workgroups."""
    wg = (torch.randn(n // 2, k, device=DEV) * 0.02).bfloat16()
    wu = (torch.randn(n // 2, k, device=DEV) * 0.02).bfloat16()
    x = torch.randn(m, k, device=DEV).bfloat16()
    ref_h = torch.nn.functional.silu(x.float() @ wg.float().t()) * (x.float() @ wu.float().t())
    wp = ops.pack_weight(ops.interleave_gate_up(torch.cat([wg, wu]), 1))
    h = ops.skinny_gemm(x, wp, nt=2, u=u)
    assert h.shape == (m, n // 2)
    _close(h.float(), ref_h, atol=3e-2, rtol=2e-2, msg="xr silu")


def test_skinny_gemm_strided_x():
    n, k, m = 512, 2048, 20
    w = (torch.randn(n, k, device=DEV) * 0.05).bfloat16()
    big = torch.randn(m, k + 512, device=DEV).bfloat16()
    x = big[:, :k]
    y = ops.skinny_gemm(x, ops.pack_weight(w), nt=2, u=-3)
    _close(y, x.float() @ w.float().t(), atol=3e-2, rtol=1e-2, msg="strided")


@pytest.mark.parametrize("hidden", [2048, 4096, 8192])
@pytest.mark.parametrize("splits", [1, 4])
def test_row_rmsnorm_from_slabs(hidden, splits):
    rows = 37
    parts = torch.randn(splits, rows, hidden, device=DEV)
    res = torch.randn(rows, hidden, device=DEV).bfloat16()
    w = (1 + 0.1 * torch.randn(hidden, device=DEV)).bfloat16()
    out = torch.empty(rows, hidden, device=DEV).bfloat16()
    x = parts.sum(0).bfloat16()
    ey, er = ref.fused_add_rmsnorm(x, res, w, 1e-5)
    ops.row_rmsnorm(out, w, 1e-5, rows, ws=parts.flatten(), splits=splits, residual=res)
    _close(res, er, atol=2e-2, rtol=1e-2, msg="residual")
    _close(out, ey, atol=3e-2, rtol=2e-2, msg="normed")


def test_slab_silu_and_store():
    rows, inter, splits = 23, 14336, 4
    parts = torch.randn(splits, rows, 2 * inter, device=DEV)
    out = torch.empty(rows, inter, device=DEV).bfloat16()
    ops.slab_silu(parts.flatten(), splits, rows, inter, out)
    _close(out, ref.silu_mul(parts.sum(0)), atol=3e-2, rtol=2e-2, msg="slab_silu")
    out2 = torch.empty(rows, 2 * inter, device=DEV).bfloat16()
    ops.slab_store(parts.flatten(), splits, rows, 2 * inter, out2)
    _close(out2, parts.sum(0), atol=3e-2, rtol=1e-2, msg="slab_store")


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (32, 8, 64)])
def test_slab_rope_kv(nq, nkv, d):
    t, bs, nblocks, splits = 19, 16, 8, 4
    cols = (nq + 2 * nkv) * d
    parts = torch.randn(splits, t, cols, device=DEV)
    pos = torch.randint(0, 4000, (t,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(d, 8192, 500000.0, None, DEV)
    slots = torch.randperm(nblocks * bs, device=DEV)[:t].int()
    k1, v1 = _alloc_cache(nblocks, nkv, bs, d)
    k2, v2 = k1.clone(), v1.clone()
    q_out = torch.zeros(t, nq * d, device=DEV).bfloat16()
    ops.slab_rope_kv(parts.flatten(), splits, t, cols, q_out, pos, cs, slots, k1, v1, nq, nkv, d)
    qkv = parts.sum(0).bfloat16()
    ref.rope_kv_write(qkv, pos, cs, slots, k2, v2, nq, nkv, d)
    _close(q_out, qkv[:, : nq * d], atol=3e-2, rtol=2e-2, msg="q")
    _close(k1, k2, atol=3e-2, rtol=2e-2, msg="k")
    _close(v1, v2, atol=3e-2, rtol=2e-2, msg="v")


@pytest.mark.parametrize("hidden", [2048, 3072, 4096, 8192])
def test_embed_rmsnorm(hidden):
    vocab = 1000
    table = torch.randn(vocab, hidden, device=DEV).bfloat16()
    w = (1 + 0.1 * torch.randn(hidden, device=DEV)).bfloat16()
    ids = torch.randint(0, vocab, (37,), dtype=torch.int32, device=DEV)
    out, res = ops.embed_rmsnorm(ids, table, w, 1e-5)
    rows = table[ids.long()]
    assert torch.equal(res, rows)
    _close(out, ref.rmsnorm(rows, w, 1e-5), atol=2e-2, rtol=1e-2, msg="embed_rmsnorm")


@pytest.mark.parametrize("n,k,splits,nt,u", [(4096, 14336, 4, 4, -3), (2048, 4096, 4, 4, -3),
                                             (128256, 4096, 1, 2, -4), (6144, 4096, 8, 2, -4),
                                             (4096, 4096, 8, 1, -4), (6144, 4096, 1, 2, -3),
                                             (28672, 4096, 1, 1, -3), (4096, 4096, 2, 2, -3),
                                             (4096, 14336, 2, 1, -3), (128256, 4096, 1, 4, -3),
                                             (4096, 14336, 7, 2, -5), (4096, 14336, 4, 1, -5),
                                             (28672, 4096, 1, 2, -5), (6144, 4096, 8, 2, -5)])
@pytest.mark.parametrize("m", [1, 37, 64])
def test_skinny_gemm_packed(m, n, k, splits, nt, u):
    """Packed-weight decode GEMMs vs fp32 torch (split-K slabs summed on the host)."""
    w = (torch.randn(n, k, device=DEV) * 0.02).bfloat16()
    x = torch.randn(m, k, device=DEV).bfloat16()
    ref_y = x.float() @ w.float().t()
    wp = ops.pack_weight(w)
    if splits == 1:
        y = ops.skinny_gemm(x, wp, splits=1, nt=nt, u=u).float()
    else:
        ws = torch.empty(splits * m * n, device=DEV)
        ops.skinny_gemm(x, wp, ws=ws, splits=splits, nt=nt, u=u)
        y = ws.view(splits, m, n).sum(0)
    _close(y, ref_y, atol=3e-2, rtol=2e-2, msg="packed skinny gemm")


# ---- fused decode layer GEMMs (csrc/kernels/skinny_pkr.hip) ------------------------

@pytest.mark.parametrize("nt,depth", [(1, 4), (2, 3), (4, 3), (4, 2)])
@pytest.mark.parametrize("m", [1, 13, 37, 64])
@pytest.mark.parametrize("splits", [1, 4])
@pytest.mark.parametrize("wn", [False, True])
def test_pkr_store(m, nt, depth, splits, wn):
    if wn and m <= 32:
        pytest.skip("wave-split-N layout is for 33-64 rows")
    n, k = 1024, 4096
    w = (torch.randn(n, k, device=DEV) * 0.02).bfloat16()
    x = torch.randn(m, k, device=DEV).bfloat16()
    wp = ops.pack_weight(w)
    ref_y = x.float() @ w.float().t()
    if splits == 1:
        out = torch.empty(m, n, device=DEV).bfloat16()
        y = ops.pkr_gemm(x, wp, out=out, nt=nt, depth=depth, wn=wn).float()
    else:
        ws = torch.empty(splits * m * n, device=DEV)
        ops.pkr_gemm(x, wp, ws=ws, splits=splits, nt=nt, depth=depth, wn=wn)
        y = ws.view(splits, m, n).sum(0)
    _close(y, ref_y, atol=3e-2, rtol=2e-2, msg="pkr store")


@pytest.mark.parametrize("m", [1, 29, 64])
@pytest.mark.parametrize("splits,nt", [(1, 2), (2, 4), (7, 2), (8, 1)])
@pytest.mark.parametrize("wn", [False, True])
def test_pkr_residual_in_launch_reduce(m, splits, nt, wn):
    """residual += x W^T with the split-K slabs reduced by the last-arriving split:
    correct, bit-identical across launches (split-order sum whoever arrives last),
    and the tickets are left re-armed."""
    if wn and m <= 32:
        pytest.skip("wave-split-N layout is for 33-64 rows")
    n, k = 2048, 14336
    w = (torch.randn(n, k, device=DEV) * 0.02).bfloat16()
    x = torch.randn(m, k, device=DEV).bfloat16()
    wp = ops.pack_weight(w)
    res0 = torch.randn(m, n, device=DEV).bfloat16()
    ws = torch.empty(splits * m * n, device=DEV)
    tickets = torch.zeros(256, dtype=torch.int32, device=DEV)
    outs = []
    for _ in range(3):
        res = res0.clone()
        ops.pkr_gemm(x, wp, "resid", residual=res, ws=ws, tickets=tickets, splits=splits, nt=nt,
                     depth=3 if nt == 2 else (4 if nt == 1 else 2), wn=wn)
        outs.append(res)
    torch.cuda.synchronize()
    assert int(tickets.abs().sum().item()) == 0
    _close(outs[0], res0.float() + x.float() @ w.float().t(), atol=5e-2, rtol=1e-2, msg="resid")
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("m", [1, 20, 64])
@pytest.mark.parametrize("nt,depth,wn", [(2, 4, False), (4, 3, False), (2, 3, True),
                                         (4, 2, True)])
def test_pkr_gate_up_silu_norm(m, nt, depth, wn):
    """RMSNorm (weight folded into W) + gate_up + SiLU-mul in one launch vs fp32."""
    if wn and m <= 32:
        pytest.skip("wave-split-N layout is for 33-64 rows")
    hidden, inter, eps = 4096, 1024, 1e-5
    wg = (torch.randn(inter, hidden, device=DEV) * 0.02).bfloat16()
    wu = (torch.randn(inter, hidden, device=DEV) * 0.02).bfloat16()
    gamma = (1 + 0.1 * torch.randn(hidden, device=DEV)).bfloat16()
    res = torch.randn(m, hidden, device=DEV).bfloat16()
    xn = ref.rmsnorm(res.float(), gamma.float(), eps)
    h_ref = torch.nn.functional.silu(xn @ wg.float().t()) * (xn @ wu.float().t())
    wgu = (torch.cat([wg, wu]).float() * gamma.float()[None, :]).bfloat16()
    wp = ops.pack_weight(ops.interleave_gate_up(wgu, nt // 2))
    h = ops.pkr_gemm(res, wp, "silu", nt=nt, depth=depth, norm=True, eps=eps, wn=wn)
    assert h.shape == (m, inter)
    _close(h, h_ref, atol=3e-2, rtol=3e-2, msg="gate_up silu norm")


def test_slab_rope_kv_residual_norm():
    """slab_rope_kv with the residual row's RMS scale (fused decode layer)."""
    nq, nkv, d = 8, 2, 128
    t, bs, nblocks, splits, hidden, eps = 11, 16, 8, 2, 2048, 1e-5
    cols = (nq + 2 * nkv) * d
    parts = torch.randn(splits, t, cols, device=DEV)
    res = torch.randn(t, hidden, device=DEV).bfloat16()
    pos = torch.randint(0, 4000, (t,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(d, 8192, 500000.0, None, DEV)
    slots = torch.randperm(nblocks * bs, device=DEV)[:t].int()
    k1, v1 = _alloc_cache(nblocks, nkv, bs, d)
    k2, v2 = k1.clone(), v1.clone()
    q_out = torch.zeros(t, nq * d, device=DEV).bfloat16()
    ops.slab_rope_kv(parts.flatten(), splits, t, cols, q_out, pos, cs, slots, k1, v1, nq, nkv, d,
                     residual=res, eps=eps)
    r = torch.rsqrt(res.float().pow(2).mean(-1, keepdim=True) + eps)
    qkv = (parts.sum(0) * r).bfloat16()
    ref.rope_kv_write(qkv, pos, cs, slots, k2, v2, nq, nkv, d)
    _close(q_out, qkv[:, : nq * d], atol=3e-2, rtol=2e-2, msg="q")
    _close(k1, k2, atol=3e-2, rtol=2e-2, msg="k")
    _close(v1, v2, atol=3e-2, rtol=2e-2, msg="v")


@pytest.mark.parametrize("m", [65, 80, 200, 256, 300, 700])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 5, 6, 10, 11, 12, 13, 14])
def test_packed_gemm_matches_fp32(m, cfg):
    """packed_gemm.hip (any M, on the decode kernels' packed image) vs fp32
    x W^T: bf16 store, split-K slabs (+ slab_store), odd N tails (N % 256 != 0)."""
    torch.manual_seed(m + cfg)
    for n, k in [(768, 512), (1040, 1024)]:
        w = (torch.randn(n, k, device="cuda") * 0.05).bfloat16()
        x = torch.randn(m, k, device="cuda").bfloat16()
        ref = x.float() @ w.float().t()
        wp = ops.pack_weight(w)
        _close(ops.packed_gemm(x, wp, cfg=cfg), ref, atol=3e-2, rtol=2e-2, msg=f"pg cfg{cfg}")
        ws = torch.empty(4 * m * n, device="cuda")
        ops.packed_gemm(x, wp, ws=ws, splits=4, epi="slab", cfg=cfg)
        out = torch.empty(m, n, device="cuda").bfloat16()
        ops.slab_store(ws, 4, m, n, out)
        _close(out, ref, atol=3e-2, rtol=2e-2, msg=f"pg cfg{cfg} split-K")


@pytest.mark.parametrize("cfg", [0, 1, 3, 5, 6, 10, 11, 12, 13, 14])
def test_packed_gemm_silu_epilogue_and_interleaved_silu(cfg):
    """gate_up in the single-image layout (interleave_gate_up(w, 1)): the GEMM's
    SiLU epilogue, silu_mul(interleaved) on its dense output and slab_silu on
    split-K slabs all equal silu(x Wg^T) * (x Wu^T)."""
    torch.manual_seed(cfg)
    inter, k, m = 1024, 512, 150
    w = (torch.randn(2 * inter, k, device="cuda") * 0.05).bfloat16()
    x = torch.randn(m, k, device="cuda").bfloat16()
    g, u = (x.float() @ w.float().t()).chunk(2, dim=-1)
    ref = torch.nn.functional.silu(g) * u
    wp = ops.pack_weight(ops.interleave_gate_up(w, 1))
    _close(ops.packed_gemm(x, wp, epi="silu", cfg=cfg), ref, atol=3e-2, rtol=2e-2, msg="silu epi")
    dense = ops.packed_gemm(x, wp, cfg=cfg)
    _close(ops.silu_mul(dense, interleaved=True), ref, atol=3e-2, rtol=2e-2, msg="silu_mul il")
    ws = torch.empty(2 * m * 2 * inter, device="cuda")
    ops.packed_gemm(x, wp, ws=ws, splits=2, epi="slab", cfg=cfg)
    h = torch.empty(m, inter, device="cuda").bfloat16()
    ops.slab_silu(ws, 2, m, inter, h, interleaved=True)
    _close(h, ref, atol=3e-2, rtol=2e-2, msg="slab_silu il")


