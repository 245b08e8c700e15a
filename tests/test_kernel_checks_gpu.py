"""Checked kernel build (SURVEY §5 "bounds checks in debug builds"):
with FT_KERNEL_CHECKS=1 ``ops.native()`` loads ``_C_checked.so``, whose attention,
RoPE/KV-write, embedding, sampler and KV-copy kernels validate every index they are
handed.  An out-of-range block-table entry, KV slot, rotary position or token id sets
the device error word (first violation: code, row, value), is clamped (no fault, no
trap), and the engine's runner turns the word into a KernelCheckError after the step.

The checks run in ONE child process (the checked extension must be the process's
``_C``); the parent only launches it and reads its verdict."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent(r"""
    import json, sys
    import torch
    sys.path.insert(0, ROOT)
    from fasttalk_llm_microservice_amd import ops
    from fasttalk_llm_microservice_amd.ops import reference as ref
    C = ops.native()
    res = {"module": C.__name__, "kernel_checks": bool(C.kernel_checks)}
    dev = "cuda"
    torch.manual_seed(0)
    nq, nkv, d, bs, nb = 8, 2, 128, 16, 8
    word = torch.zeros(4, dtype=torch.int32, device=dev)
    C.set_kernel_checks(word)

    def take():
        torch.cuda.synchronize()
        w = word.cpu().tolist()
        word.zero_()
        return w

    k = torch.randn(nb, nkv, bs, d, device=dev).bfloat16()
    v = torch.randn(nb, nkv, d, bs, device=dev).bfloat16()
    lens = [40, 17]
    bt = torch.tensor([[3, 5, 1], [6, 2, 0]], dtype=torch.int32, device=dev)
    sl = torch.tensor(lens, dtype=torch.int32, device=dev)
    q = torch.randn(2, nq * d, device=dev).bfloat16()
    n_out, n_ml = ops.decode_workspace(2, nq, nkv, d)
    tmp_out = torch.empty(n_out, device=dev)
    tmp_ml = torch.empty(n_ml, device=dev)
    out = torch.empty(2, nq * d, device=dev).bfloat16()
    ops.decode_attention(out, q, k, v, bt, sl, tmp_out, tmp_ml, nq, nkv, d, d ** -0.5)
    expect = ref.paged_attention(q.view(2, nq, d), k, v, bt, sl,
                                 torch.arange(3, dtype=torch.int32), d ** -0.5).view(2, nq * d)
    res["valid_word"] = take()
    res["valid_err"] = (out.float() - expect.float()).abs().max().item()

    # a CPU-constructed block table with an entry past the pool (9999 >= 8 blocks)
    bad = torch.tensor([[3, 9999, 1], [6, 2, 0]], dtype=torch.int32).to(dev)
    ops.decode_attention(out, q, k, v, bad, sl, tmp_out, tmp_ml, nq, nkv, d, d ** -0.5)
    res["bad_bt_word"] = take()
    res["bad_bt_finite"] = bool(torch.isfinite(out.float()).all())

    # RoPE + KV write: a position past the 64-row rotary table, a slot past 8 x 16
    cs = ref.rope_cos_sin(d, 64, 500000.0, None, dev)
    qkv = torch.randn(3, (nq + 2 * nkv) * d, device=dev).bfloat16()
    pos = torch.tensor([1, 2, 3], dtype=torch.int32, device=dev)
    slots = torch.tensor([0, 5, -1], dtype=torch.int32, device=dev)
    ops.rope_kv_write(qkv.clone(), pos, cs, slots, k, v, nq, nkv, d)
    res["rope_ok_word"] = take()
    ops.rope_kv_write(qkv.clone(), torch.tensor([1, 500, 3], dtype=torch.int32, device=dev),
                      cs, slots, k, v, nq, nkv, d)
    res["bad_pos_word"] = take()
    ops.rope_kv_write(qkv.clone(), pos, cs, torch.tensor([0, 8 * 16 + 5, -1], dtype=torch.int32,
                      device=dev), k, v, nq, nkv, d)
    res["bad_slot_word"] = take()

    # embedding: id 5000 >= vocab 1000 (the kernel clamps it; the word reports it)
    table = torch.randn(1000, 2048, device=dev).bfloat16()
    w = torch.ones(2048, device=dev).bfloat16()
    ops.embed_rmsnorm(torch.tensor([7, 5000], dtype=torch.int32, device=dev), table, w, 1e-5)
    res["bad_id_word"] = take()

    # KV block copy with a destination past the pool
    ops.kv_block_copy(k, v, torch.tensor([[1, 42]], dtype=torch.int32, device=dev))
    res["bad_copy_word"] = take()

    # the engine path: a clean generate, then a step whose block table is corrupted
    # on the host turns into KernelCheckError from the runner
    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.runner import KernelCheckError
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
    eng = LLMEngine(EngineConfig(model="tiny", device="cuda", num_kv_blocks=64,
                                 max_model_len=512, max_num_seqs=4))
    r = eng.runner
    outs = eng.generate([[1, 2, 3, 4, 5]], SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))
    res["engine_clean"] = [len(o) for o in outs]
    res["engine_clean_word"] = r.d_check.cpu().tolist()
    orig = r._decode_fill

    def corrupt(seqs, nb_, st):
        m = orig(seqs, nb_, st)
        st.hbt[0, 0] = 10 ** 6      # past the 64-block pool
        return m
    r._decode_fill = corrupt
    try:
        eng.generate([[9, 8, 7, 6]], SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))
        res["engine_raised"] = None
    except KernelCheckError as e:
        res["engine_raised"] = [e.code, e.value]
    # the word is cleared as the error is raised: the next clean request succeeds
    r._decode_fill = orig
    eng.fail_unfinished("kernel check", reset_cache=True)   # what the serving loop does
    eng.runner.kernel_check()
    outs = eng.generate([[3, 1, 4, 1, 5]], SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))
    res["engine_after"] = [len(o) for o in outs]
    res["engine_after_word"] = r.d_check.cpu().tolist()
    print("RESULT " + json.dumps(res), flush=True)
""")


def test_checked_build_catches_out_of_range_indices():
    env = dict(os.environ, FT_KERNEL_CHECKS="1", FT_AUTOBUILD="0")
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert r.returncode == 0 and lines, (r.stdout[-3000:], r.stderr[-3000:])
    res = json.loads(lines[-1][len("RESULT "):])
    assert res["module"].endswith("_C_checked") and res["kernel_checks"], res
    # valid inputs: no report, correct numerics
    assert res["valid_word"][0] == 0 and res["valid_err"] < 3e-2, res
    assert res["rope_ok_word"][0] == 0, res
    # each violation: counted, first code / value recorded, kernel did not fault
    assert res["bad_bt_word"][0] > 0 and res["bad_bt_word"][1] == 1 and res["bad_bt_word"][3] == 9999, res
    assert res["bad_bt_finite"], res
    assert res["bad_pos_word"][1] == 3 and res["bad_pos_word"][3] == 500, res
    assert res["bad_slot_word"][1] == 2 and res["bad_slot_word"][3] == 8 * 16 + 5, res
    assert res["bad_id_word"][1] == 4 and res["bad_id_word"][3] == 5000, res
    assert res["bad_copy_word"][1] == 6 and res["bad_copy_word"][3] == 42, res
    assert "[ft-check]" in r.stdout + r.stderr
    # engine: clean run leaves the word at zero; a corrupted step raises KernelCheckError
    assert res["engine_clean"] == [4] and res["engine_clean_word"][0] == 0, res
    assert res["engine_raised"] == [1, 10 ** 6], res
    assert res["engine_after"] == [4] and res["engine_after_word"][0] == 0, res
