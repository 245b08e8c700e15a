"""Decode GEMM plan tables of the Llama model (models/llama.py): bucket lookup,
the shape fallbacks of the fused plan, the FT_PACKED_PLAN overlay and the
fused_plan.json loader.  CPU only: no kernel runs."""
import copy
import json

import pytest

from fasttalk_llm_microservice_amd.models import llama


@pytest.fixture
def plans():
    saved = copy.deepcopy(llama.PACKED_PLAN), copy.deepcopy(llama.FUSED_PLAN)
    yield
    llama.PACKED_PLAN.clear()
    llama.PACKED_PLAN.update(saved[0])
    llama.FUSED_PLAN.clear()
    llama.FUSED_PLAN.update(saved[1])


def test_buckets_round_up():
    assert llama.fused_bucket(1) == 1
    assert llama.fused_bucket(9) == 16
    assert llama.fused_bucket(33) == 48
    assert llama.fused_bucket(50) == 64
    assert llama.packed_cfg("o", 65) is None  # above PACKED_ROWS: packed_gemm.hip


def test_packed_overlay_sets_and_removes(plans):
    llama._overlay_packed_plan(json.dumps({"qkv": {"64": [4, -3, 2]}, "lm": {"32": []},
                                           "nope": {"8": [1, -3, 1]}}))
    assert llama.PACKED_PLAN["qkv"][64] == (4, -3, 2)
    assert 32 not in llama.PACKED_PLAN["lm"]
    assert "nope" not in llama.PACKED_PLAN
    assert llama.packed_cfg("qkv", 50) == (4, -3, 2)


def test_packable_follows_plan(plans):
    assert llama._packable(6144, 4096, "qkv")
    llama.PACKED_PLAN["qkv"][64] = (4, -4, 16)  # K step 512 * 16 does not divide 4096
    assert not llama._packable(6144, 4096, "qkv")


def test_fused_cfg_shape_fallbacks(plans):
    llama.FUSED_PLAN["down"][64] = (4, 2, 4, 1)
    assert llama.fused_cfg("down", 50, 4096, 14336) == (4, 2, 4, True)
    # K not divisible by 64 * splits -> one split; N not tiling 16 * nt -> nt 1
    assert llama.fused_cfg("down", 50, 4096, 14336 - 64)[2] == 1
    nt, depth, _, wn = llama.fused_cfg("down", 50, 4096 + 16, 14336)
    assert (nt, depth, wn) == (1, 2, False)
    # wave-split-N only above 32 rows
    assert llama.fused_cfg("down", 16, 4096, 14336)[3] is False


def test_fused_plan_loader_validates(plans, tmp_path):
    p = tmp_path / "plan.json"
    p.write_text(json.dumps({"o": {"8": [2, 2, 2, 0], "7": [1, 2, 1, 0]},
                             "down": {"16": [1, 2, 99, 0]}}))
    before_down = llama.FUSED_PLAN["down"][16]
    llama.load_fused_plan(str(p))
    assert llama.FUSED_PLAN["o"][8] == (2, 2, 2, 0)
    assert 7 not in llama.FUSED_PLAN["o"]  # not a bucket
    assert llama.FUSED_PLAN["down"][16] == before_down  # splits out of range


def test_prefill_split_plan_covers_ranges():
    """ops.build_prefill_tiles: every query block's KV tiles are covered exactly
    once by its items; split blocks get consecutive partial slots listed in the
    combine entries; short histories and an exhausted slot budget stay unsplit."""
    from fasttalk_llm_microservice_amd import ops

    q_lens = [100, 37, 64, 130, 3, 1]
    seq_lens = [3000, 4037, 64, 830, 1503, 64]
    items, comb = ops.build_prefill_tiles(q_lens, 64, seq_lens=seq_lens, nkv=8, num_cus=256)
    assert comb and len(items) > 7
    by_block = {}
    for b, s, rng, slot in items:
        by_block.setdefault((b, s), []).append((rng >> 16, rng & 0xFFFF, slot))
    for (b, s), parts in by_block.items():
        L, ql = seq_lens[b], q_lens[b]
        nkt = -(-min(L, L - ql + s + min(64, ql - s)) // 64)
        if len(parts) == 1:
            assert parts[0] == (0, 0xFFFF, -1)
            continue
        parts.sort()
        assert parts[0][0] == 0 and parts[-1][1] == nkt
        assert all(a[1] == c[0] and a[0] < a[1] for a, c in zip(parts, parts[1:]))
        (cb,) = [c for c in comb if (c[0], c[1]) == (b, s)]
        assert [p[2] for p in parts] == list(range(cb[2], cb[2] + cb[3]))
    # no seq_lens: one item per query block, nothing to combine
    items, comb = ops.build_prefill_tiles(q_lens, 64)
    assert comb == [] and all(r == 0xFFFF and sl == -1 for _, _, r, sl in items)
    # slot budget: blocks that would exceed it run unsplit
    items, comb = ops.build_prefill_tiles(q_lens, 64, seq_lens=seq_lens, num_cus=256, max_partials=4)
    assert sum(c[3] for c in comb) <= 4


def test_prefill_split_plan_fills_whole_rounds():
    """The prefill kernel runs one workgroup per CU, so the plan counts rounds of
    num_cus workgroups: 5 prompts x 107 new tokens over 3k cached fit ONE round
    (the old ~2-per-CU target gave 520 workgroups: a third round for 8 of them),
    and no plan's estimated makespan is worse than the round-blind split's."""
    from fasttalk_llm_microservice_amd import ops

    items, comb = ops.build_prefill_tiles([107] * 5, 64, seq_lens=[3107] * 5, nkv=8, num_cus=256)
    assert len(items) * 8 <= 256 and comb
    for S, Q, C in [(10, 100, 3000), (4, 128, 3000), (1, 512, 3000), (50, 60, 3000), (3, 300, 5000)]:
        items, comb = ops.build_prefill_tiles([Q] * S, 64, seq_lens=[Q + C] * S, nkv=8, num_cus=256)
        lens = [((r & 0xFFFF) - (r >> 16)) if r != 0xFFFF else None for _, _, r, _ in items]
        assert sum(c[3] for c in comb) <= ops.PREFILL_MAX_PARTIALS
        rounds = -(-len(items) * 8 // 256)
        assert rounds <= ops.PREFILL_MAX_ROUNDS
        if any(lens):
            longest = max(x for x in lens if x)
            # round-blind plan: ~64 items of ceil(total / 64) tiles, rounded up per block
            nblocks = S * -(-Q // 64)
            total = sum(-(-min(Q + C, C + s + min(64, Q - s)) // 64) for s in range(0, Q, 64)) * S
            blind = max(4, -(-total // 64))
            blind_items = sum(-(-min(Q + C, C + s + min(64, Q - s)) // 64 // blind) or 1
                              for s in range(0, Q, 64)) * S
            assert rounds * (longest + 1) <= -(-max(blind_items, nblocks) * 8 // 256) * (blind + 1) + 1


def test_prefill_fixed_chunk_plan_is_absolute():
    """Batch-invariant prefill plan (fixed_chunk): a block's KV range is cut at
    absolute multiples of the chunk, whatever the other blocks of the step, so the
    same query rows see the same pieces in any batch; it never silently falls back
    to an unsplit item when the partial slots run out."""
    from fasttalk_llm_microservice_amd import ops

    C = 4
    a, comb_a = ops.build_prefill_tiles([100], 64, seq_lens=[3000], fixed_chunk=C)
    b, comb_b = ops.build_prefill_tiles([37, 100, 5], 64, seq_lens=[900, 3000, 4000], fixed_chunk=C)
    ranges = lambda items, seq: sorted((s, r >> 16, r & 0xFFFF) for bb, s, r, _ in items if bb == seq)
    assert ranges(a, 0) == ranges(b, 1)
    for s, lo, hi in ranges(a, 0):
        assert lo % C == 0 and (hi - lo == C or hi == -(-min(3000, 2900 + s + min(64, 100 - s)) // 64))
    assert [c[3] for c in comb_a] == [c[3] for c in comb_b if c[0] == 1]
    with pytest.raises(RuntimeError):
        ops.build_prefill_tiles([100] * 8, 64, seq_lens=[3000] * 8, fixed_chunk=C, max_partials=8)
    # no seq_lens (CPU path): nothing is split
    items, comb = ops.build_prefill_tiles([100], 64, fixed_chunk=C)
    assert comb == [] and all(r == 0xFFFF for _, _, r, _ in items)


def test_decode_workspace_piece_mode_slots():
    """Piece mode needs one partial slot per piece of the longest sequence."""
    from fasttalk_llm_microservice_amd import ops

    n_out, n_ml = ops.decode_workspace(4, 32, 8, 128, waves=16, piece=32, max_len=2048)
    assert n_out == 4 * 8 * 4 * 4 * 128 and n_ml == 4 * 8 * 4 * 4 * 2   # 128 tiles -> 4 pieces
    n0, _ = ops.decode_workspace(4, 32, 8, 128, waves=16)
    assert n0 == (4 * 8 + 16) * 4 * 128


def test_w4_plan_uses_mh_above_48_rows():
    """49..64 rows run the "mh" W4 kernel for qkv / o / gate_up (xr 4 / 5), down
    and smaller batches keep the round-5 entries; every entry tiles the Llama-3-8B
    shapes, and w4_fits rejects shapes a TP shard can break."""
    assert llama.w4_cfg("qkv", 50) == (2, 4, 4)
    assert llama.w4_cfg("gu", 64) == (2, 1, 5)
    assert llama.w4_cfg("down", 50) == llama.W4_PLAN["down"][64]
    assert llama.w4_cfg("qkv", 40) == llama.W4_PLAN["qkv"][64]
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336)}
    for proj, (n, k) in shapes.items():
        for rows in (1, 8, 16, 20, 33, 48, 50, 64):
            nt, sp, xr = llama.w4_cfg(proj, rows)
            assert llama.w4_fits(xr, nt, sp, n, k), (proj, rows)
    assert not llama.w4_fits(4, 2, 4, 6144 // 8 + 16, 4096)   # N % 32
    assert not llama.w4_fits(4, 2, 1, 4096, 14336)            # K slice > 4096 (x-sum table)
    assert not llama.w4_fits(1, 2, 1, 96, 4096)               # xr: N % 128
    # Llama-3-70B (TP=1): gate_up's K 8192 is past mh's one-split K slice -> the xr
    # SiLU entry of the bucket plan, not the register kernel
    assert llama.w4_cfg("gu", 50, 57344, 8192) == llama.W4_PLAN["gu"][64]
    assert llama.w4_cfg("qkv", 50, 10240, 8192) == (2, 8, 4)   # the wide (70B) entries
    assert llama.w4_cfg("o", 50, 8192, 8192) == (4, 2, 0)
    assert llama.w4_cfg("qkv", 50, 6144, 4096) == (2, 4, 4)
    assert llama.w4_cfg("down", 50, 8192, 28672) == llama.W4_PLAN["down"][64]
