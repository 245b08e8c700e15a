"""fp8 (e4m3) KV cache (ENGINE_KV_CACHE_DTYPE=fp8): the KV8 paths of the gfx950
kernels that write (rope_kv.hip, fused_epilogue.hip slab_rope_kv) and read
(attn_decode.hip, attn_prefill.hip) the paged cache, and the byte copies
(kv_copy.hip), against the fp32 PyTorch reference on the same cache contents (an
fp8 value widens to bf16 exactly, so the reference sees the bytes the kernels
read)."""
import pytest
import torch

from fasttalk_llm_microservice_amd import ops
from fasttalk_llm_microservice_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
F8 = torch.float8_e4m3fn


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


def _f8(x):
    return x.float().clamp(-448, 448).to(F8)


def _alloc_cache(nblocks, nkv, bs, d, scale=1.0):
    """fp8 K blocks [nkv, bs, d] and transposed V blocks [nkv, d, bs]."""
    k = _f8(torch.randn(nblocks, nkv, bs, d, device=DEV) * scale)
    v = _f8(torch.randn(nblocks, nkv, d, bs, device=DEV) * scale)
    return k, v


def _bf(c):
    return c.to(torch.bfloat16)


def _bytes(c):
    return c.view(torch.uint8)


def test_fp8_roundtrip_matches_torch():
    """The kernels' converters are OCP e4m3 (torch.float8_e4m3fn): a cache written
    by rope_kv_write from values already on the fp8 grid holds them bit-exactly,
    including values past the format's range (clamped to +-448, not NaN)."""
    nq, nkv, d, t, bs = 8, 8, 128, 16, 16
    qkv = torch.zeros(t, (nq + 2 * nkv) * d, device=DEV).bfloat16()
    grid = _f8(torch.randn(t, nkv * d, device=DEV) * 20)
    vals = grid.float()
    vals[0, :4] = torch.tensor([1000.0, -1000.0, 448.0, 0.0], device=DEV)
    qkv[:, (nq + nkv) * d:] = vals.bfloat16()
    pos = torch.zeros(t, dtype=torch.int32, device=DEV)
    cs = ref.rope_cos_sin(d, 64, 500000.0, None, DEV)
    slots = torch.arange(t, dtype=torch.int32, device=DEV)
    k, v = _alloc_cache(1, nkv, bs, d)
    ops.rope_kv_write(qkv, pos, cs, slots, k, v, nq, nkv, d)
    got = v[0].float().permute(2, 0, 1).reshape(t, nkv * d)     # V^T blocks -> token rows
    want = _f8(vals.bfloat16()).float()
    assert torch.equal(got.cpu(), want.cpu())
    assert got[0, 0].item() == 448.0 and got[0, 1].item() == -448.0


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (32, 8, 64), (8, 1, 128)])
def test_fp8_rope_kv_write(nq, nkv, d):
    t, bs, nblocks = 45, 16, 20
    qkv = (torch.randn(t, (nq + 2 * nkv) * d, device=DEV) * 3).bfloat16()
    pos = torch.randint(0, 4000, (t,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(d, 8192, 500000.0, None, DEV)
    slots = torch.randperm(nblocks * bs, device=DEV)[:t].int()
    slots[3] = -1
    k1, v1 = _alloc_cache(nblocks, nkv, bs, d)
    k2, v2 = k1.clone(), v1.clone()
    q1, q2 = qkv.clone(), qkv.clone()
    ops.rope_kv_write(q1, pos, cs, slots, k1, v1, nq, nkv, d)
    ref.rope_kv_write(q2, pos, cs, slots, k2, v2, nq, nkv, d)
    _close(q1[:, : nq * d], q2[:, : nq * d], atol=2e-2, rtol=1e-2, msg="q")
    # K: the kernel rounds fp32 -> fp8 once, the reference via bf16 (double rounding can
    # land one e4m3 step away: up to 1/8 relative)
    _close(k1, k2, atol=2e-3, rtol=0.126, msg="k cache")
    assert (k1.float() != k2.float()).float().mean().item() < 0.01
    assert torch.equal(_bytes(v1), _bytes(v2))   # V: bf16 -> fp8, one rounding on both sides


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (32, 8, 64)])
def test_fp8_slab_rope_kv(nq, nkv, d):
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
    # the reference rounds the slab sum to bf16 before RoPE (the bf16 test's 3e-2, which
    # cancellation in x1 cos - x2 sin turns into absolute error), then one e4m3 step
    _close(k1, k2, atol=3e-2, rtol=0.126, msg="k")
    _close(v1, v2, atol=3e-2, rtol=0.126, msg="v")


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


def _decode_case(lens, nq, nkv, d, bs=16, fused=True, piece=0, calls=2):
    nblocks = sum((l + bs - 1) // bs for l in lens) + 4
    k, v = _alloc_cache(nblocks, nkv, bs, d)
    bt = _random_tables(lens, bs, nblocks).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    b = len(lens)
    q = torch.randn(b, nq * d, device=DEV).bfloat16()
    n_out, n_ml = ops.decode_workspace(b, nq, nkv, d, piece=piece, max_len=max(lens))
    tmp_out = torch.full((n_out,), float("nan"), device=DEV)
    tmp_ml = torch.full((n_ml,), float("nan"), device=DEV)
    out = torch.full((b, nq * d), float("nan"), device=DEV).bfloat16()
    scale = d ** -0.5
    cnt = ops.decode_counters(b, nkv, DEV) if (fused or piece) else None
    for _ in range(calls):
        first = out.clone()
        ops.decode_attention(out, q, k, v, bt, sl, tmp_out, tmp_ml, nq, nkv, d, scale, counters=cnt,
                             piece=piece)
    if calls > 1:
        assert torch.equal(first, out)
    if cnt is not None:
        torch.cuda.synchronize()
        assert int(cnt.abs().sum()) == 0, "combine tickets must be left zeroed"
    expect = ref.paged_attention(q.view(b, nq, d), _bf(k), _bf(v), bt, sl,
                                 torch.arange(b + 1, dtype=torch.int32), scale).view(b, nq * d)
    return out, expect


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (64, 8, 128), (8, 8, 128), (24, 8, 128),
                                      (32, 8, 64), (8, 1, 128)])
@pytest.mark.parametrize("fused", [True, False])
def test_fp8_decode_attention(nq, nkv, d, fused):
    out, expect = _decode_case([1, 17, 255, 256, 257, 1000, 2100], nq, nkv, d, fused=fused)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="fp8 decode attention")


@pytest.mark.parametrize("b,max_len", [(1, 8192), (50, 6000), (64, 8192)])
def test_fp8_decode_attention_serving_shapes(b, max_len):
    g = torch.Generator().manual_seed(b)
    lens = torch.randint(max(1, max_len // 4), max_len + 1, (b,), generator=g).tolist()
    lens[0] = max_len
    out, expect = _decode_case(lens, 32, 8, 128)
    assert torch.isfinite(out.float()).all()
    _close(out, expect, atol=2e-2, rtol=2e-2, msg=f"fp8 decode attention b={b}")


def test_fp8_decode_attention_batch_invariant_pieces():
    out, expect = _decode_case([5, 600, 1500, 33], 32, 8, 128, piece=ops.DECODE_INV_PIECE)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="fp8 decode attention (pieces)")


@pytest.mark.parametrize("bs", [32, 64])
def test_fp8_decode_attention_block_sizes(bs):
    out, expect = _decode_case([5, 64, 300, 1025], 32, 8, 128, bs=bs)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg=f"fp8 decode attention bs={bs}")


def _prefill_run(seqs, nq, nkv, d, split, bs=16, invariant=False):
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
                                          seq_lens=lens if split else None, nkv=nkv, num_cus=256,
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
                              po, pml, cb, len(comb), sum(c[3] for c in comb), invariant=invariant)
    else:
        ops.prefill_attention(out, q, k, v, bt, sl, qsl.to(DEV), ti, len(tiles), nq, nkv, d, scale,
                              invariant=invariant)
    expect = ref.paged_attention(q.view(t, nq, d), _bf(k), _bf(v), bt, sl, qsl, scale).view(t, nq * d)
    return out, expect


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (24, 8, 128), (64, 8, 128), (32, 8, 64),
                                      (8, 8, 128)])
@pytest.mark.parametrize("invariant", [False, True])
def test_fp8_prefill_attention(nq, nkv, d, invariant):
    # (new tokens, cached prefix): tile / block edges, one-tile and many-tile ranges
    seqs = [(1, 0), (5, 0), (64, 0), (77, 33), (16, 300), (130, 1), (3, 500), (40, 23)]
    out, expect = _prefill_run(seqs, nq, nkv, d, split=False, invariant=invariant)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="fp8 prefill attention")


@pytest.mark.parametrize("nq,nkv,d", [(32, 8, 128), (32, 8, 64)])
def test_fp8_prefill_attention_split_kv(nq, nkv, d):
    seqs = [(100, 2900), (37, 4000), (64, 0), (130, 700), (3, 1500), (1, 63)]
    out, expect = _prefill_run(seqs, nq, nkv, d, split=True)
    assert torch.isfinite(out.float()).all()
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="fp8 prefill attention split-KV")


def test_fp8_prefill_attention_block_size_32():
    out, expect = _prefill_run([(50, 70), (9, 200)], 32, 8, 128, split=False, bs=32)
    _close(out, expect, atol=2e-2, rtol=2e-2, msg="fp8 prefill attention bs=32")


def test_fp8_kv_block_copy_and_swap():
    k, v = _alloc_cache(10, 8, 16, 128)
    k0, v0 = k.clone(), v.clone()
    pairs = torch.tensor([[1, 5], [2, 7]], dtype=torch.int32, device=DEV)
    ops.kv_block_copy(k, v, pairs)
    assert torch.equal(_bytes(k[5]), _bytes(k0[1])) and torch.equal(_bytes(v[7]), _bytes(v0[2]))
    assert torch.equal(_bytes(k[0]), _bytes(k0[0]))
    layers = [_alloc_cache(12, 8, 16, 128) for _ in range(3)]
    ptrs = torch.tensor([c.data_ptr() for kv in layers for c in kv], dtype=torch.int64, device=DEV)
    be = 8 * 16 * 128
    ids = torch.tensor([7, 0, 11, 3], dtype=torch.int32, device=DEV)
    st = torch.empty(4, 6 * be, dtype=F8, device=DEV)
    ops.kv_swap(layers, ptrs, ids, st, to_staging=True)
    expect = torch.stack([torch.cat([_bytes(c[b]).flatten() for kv in layers for c in kv])
                          for b in ids.tolist()])
    assert torch.equal(_bytes(st), expect)
    new = _f8(torch.randn(2, 6 * be, device=DEV))
    ids2 = torch.tensor([5, 9], dtype=torch.int32, device=DEV)
    ops.kv_swap(layers, ptrs, ids2, new, to_staging=False)
    flat = [c for kv in layers for c in kv]
    for ci, c in enumerate(flat):
        for i, b in enumerate((5, 9)):
            assert torch.equal(_bytes(c[b]).flatten(), _bytes(new[i, ci * be:(ci + 1) * be]))
