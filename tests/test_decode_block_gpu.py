"""Persistent post-attention decode block (csrc/kernels/decode_block.hip) against the
fp32 PyTorch reference of the same three steps:

    r1 = residual + attn Wo^T                      (bf16 residual stream)
    h  = silu(g) * u,  [g | u] = rmsnorm(r1; ln2) [Wg | Wu]^T
    r2 = r1 + h Wd^T

at Llama-3-8B layer shapes, 1..64 rows; plus the launch contract: counters left
zeroed, no give-up flag, bit-identical relaunches and hipGraph replay."""
import pytest
import torch

from fasttalk_llm_microservice_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, KO, INTER, EPS = 4096, 4096, 14336, 1e-5


def _close(a, b, atol, rtol, msg):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).sum().item()
    assert bad == 0, f"{msg}: {bad} elems out of tol, max err {err.max().item():.4g}"


@pytest.fixture(scope="module")
def layer():
    ops.native()
    if ops.decode_block_plan(H, KO, INTER) is None:
        pytest.skip("decode block geometry does not fit this device")
    g = torch.Generator(device=DEV).manual_seed(7)
    wo = (torch.randn(H, KO, device=DEV, generator=g) * 0.02).bfloat16()
    wg = (torch.randn(INTER, H, device=DEV, generator=g) * 0.02).bfloat16()
    wu = (torch.randn(INTER, H, device=DEV, generator=g) * 0.02).bfloat16()
    wd = (torch.randn(H, INTER, device=DEV, generator=g) * 0.02).bfloat16()
    gamma = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).bfloat16()
    wgu_f = (torch.cat([wg, wu]).float() * gamma.float()[None, :]).bfloat16()   # ln2 folded
    pk = dict(wo=ops.pack_weight(wo), wgu=ops.pack_weight(ops.interleave_gate_up(wgu_f, 1)),
              wd=ops.pack_weight(wd))
    return dict(wo=wo, wgu_f=wgu_f, wd=wd, pk=pk)


def _scratch(m):
    ws = torch.empty(ops.decode_block_ws_floats(H, m), device=DEV)
    so, sd, tpw, grid = ops.decode_block_plan(H, KO, INTER)
    xg = torch.empty((grid // 2) * 2 * 4 * 256, device=DEV)
    ctl = torch.zeros(ops.decode_block_ctl_words(), dtype=torch.int32, device=DEV)
    h = torch.empty(64, INTER, dtype=torch.bfloat16, device=DEV)
    return ws, xg, ctl, h


def _reference(attn, res, L):
    r1 = (res.float() + attn.float() @ L["wo"].float().t()).bfloat16().float()
    rs = torch.rsqrt(r1.pow(2).mean(-1, keepdim=True) + EPS)
    gu = (r1 @ L["wgu_f"].float().t()) * rs
    h = (torch.nn.functional.silu(gu[:, :INTER]) * gu[:, INTER:]).bfloat16().float()
    r2 = r1 + h @ L["wd"].float().t()
    return r1, h, r2


@pytest.mark.parametrize("m", [1, 16, 33, 40, 50, 64])
def test_decode_block_matches_fp32(layer, m):
    torch.manual_seed(m)
    attn = torch.randn(m, KO, device=DEV).bfloat16()
    res0 = torch.randn(m, H, device=DEV).bfloat16()
    ws, xg, ctl, h = _scratch(m)
    res = res0.clone()
    pk = layer["pk"]
    ops.decode_block(attn, res, h, pk["wo"], pk["wgu"], pk["wd"], ws, xg, ctl, EPS)
    torch.cuda.synchronize()
    r1, h_ref, r2 = _reference(attn, res0, layer)
    assert int(ctl.abs().sum().item()) == 0, ctl.nonzero().flatten().tolist()
    _close(h[:m], h_ref, atol=3e-2, rtol=3e-2, msg="h")
    _close(res, r2, atol=6e-2, rtol=2e-2, msg="residual")


def test_decode_block_relaunch_and_graph(layer):
    """Counters re-armed by the kernel itself: eager relaunches and a captured graph
    replayed several times give bit-identical residuals (split-order combines)."""
    m = 50
    attn = torch.randn(m, KO, device=DEV).bfloat16()
    res0 = torch.randn(m, H, device=DEV).bfloat16()
    ws, xg, ctl, h = _scratch(m)
    pk = layer["pk"]
    outs = []
    for _ in range(3):
        res = res0.clone()
        ops.decode_block(attn, res, h, pk["wo"], pk["wgu"], pk["wd"], ws, xg, ctl, EPS)
        outs.append(res)
    res_g = res0.clone()
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        with torch.cuda.graph(graph, stream=stream):
            ops.decode_block(attn, res_g, h, pk["wo"], pk["wgu"], pk["wd"], ws, xg, ctl, EPS)
    torch.cuda.current_stream().wait_stream(stream)
    for _ in range(4):
        res_g.copy_(res0)
        graph.replay()
    torch.cuda.synchronize()
    assert int(ctl.abs().sum().item()) == 0
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert torch.equal(outs[0], res_g)
