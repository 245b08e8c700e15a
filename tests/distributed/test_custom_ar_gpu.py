"""Custom one-shot all-reduce (csrc/kernels/custom_ar.hip) with two ranks that
share ONE MI355X: two processes, IPC-mapped uncached regions of the same device,
the same signalling protocol the TP group runs over xGMI.  Checks sums against a
fp32 host reference, eager and captured in a hipGraph (fixed kernel arguments,
epochs advance on the device), and that no wait ran out of spin budget."""
import multiprocessing as mp
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(trial, world, n):
    import torch

    return [torch.randn(n, generator=torch.Generator().manual_seed(1000 * trial + r)).bfloat16()
            for r in range(world)]


def _worker(rank, world, port, q):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    import torch
    import torch.distributed as dist

    from fasttalk_llm_microservice_amd.parallel.custom_allreduce import CustomAllReduce

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    ar = CustomAllReduce(dist.group.WORLD, rank, world, torch.device("cuda:0"),
                         max_bytes=1 << 20, spin_budget=1 << 24)
    errs = []
    for trial, n in enumerate([64 * 4096, 8 * 4096, 4096, 50 * 4096]):
        xs = _inputs(trial, world, n)
        expect = sum(x.float() for x in xs)
        x = xs[rank].cuda()
        ar.all_reduce(x)
        torch.cuda.synchronize()
        errs.append((x.float().cpu() - expect).abs().max().item())
    # hipGraph: the same kernel replayed with new data in the captured buffer
    n = 16 * 4096
    buf = torch.zeros(n, device="cuda").bfloat16()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.all_reduce(buf)  # warm-up call (both ranks make it)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ar.all_reduce(buf)
    for trial in range(10, 14):
        xs = _inputs(trial, world, n)
        buf.copy_(xs[rank].cuda())
        g.replay()
        torch.cuda.synchronize()
        errs.append((buf.float().cpu() - sum(x.float() for x in xs)).abs().max().item())
    q.put((rank, errs, ar.healthy()))
    dist.barrier()
    ar.close()
    dist.destroy_process_group()


def test_custom_allreduce_two_ranks_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, errs, healthy in results:
        assert healthy, f"rank {rank}: a wait ran out of spin budget"
        assert max(errs) < 0.06, f"rank {rank}: max abs err {max(errs)} ({errs})"
