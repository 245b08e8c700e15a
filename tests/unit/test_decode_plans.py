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
    assert llama.packed_cfg("o", 65) is None  # above PACKED_ROWS: the library GEMM


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
