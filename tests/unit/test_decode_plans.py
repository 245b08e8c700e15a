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
