"""The data-parallel gradient exchange (GradientBuckets) captured in a HIP graph with
its RCCL all-reduce, as bench.py's N > 1 layer step replays it.

Only one GPU is available here, so the process group is a world-size-1 RCCL ("nccl") group and
GradientBuckets is told the world has 2 ranks: every collective still runs through RCCL on the
capturing stream, the flags / averaging / in-place views are the N > 1 code path, and the
expected result is the local gradient / 2 (one rank's sum, averaged over "2"). Multi-rank values
are covered on CPU by tests/test_distributed.py (gloo)."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_world1(device):
    fd, path = tempfile.mkstemp(prefix="protoseg_rccl_")
    os.close(fd)
    os.unlink(path)
    dist.init_process_group("nccl", init_method=f"file://{path}", rank=0, world_size=1,
                            device_id=device)
    try:
        yield
    finally:
        dist.destroy_process_group()


def test_exchange_captured_with_rccl(device, rccl_world1, monkeypatch):
    from protoseg_amd.distributed import GradientBuckets
    from protoseg_amd.optim import Adam
    gen = torch.Generator().manual_seed(1)
    params = [torch.nn.Parameter(torch.rand(361, 64, generator=gen).to(device)),
              torch.nn.Parameter(torch.rand(19, 361, generator=gen).to(device))]
    gb = GradientBuckets(params, average=True)
    monkeypatch.setattr(gb, "_world", lambda: 2)
    for p in params:
        p.grad = torch.zeros_like(p)
    gb.bind_grads()
    opt = Adam(params, lr=1e-3)
    src = [torch.rand(p.shape, generator=gen).to(device) for p in params]
    ref_params = [p.detach().clone() for p in params]

    def step():
        for p, s in zip(params, src):
            p.grad.copy_(s)          # what the layer backward writes into the bound views
        gb.allreduce()
        gb.wait()
        opt.step()

    stream = torch.cuda.Stream(device)
    with torch.cuda.stream(stream):
        step()  # eager warm-up (allocates the optimizer state)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            step()
        for p, r in zip(params, ref_params):
            p.data.copy_(r)
        for _ in range(3):
            g.replay()
    torch.cuda.synchronize()
    for p, s in zip(params, src):
        assert torch.equal(p.grad, s / 2)  # reduced in place, averaged over the "2" ranks
        assert any(f.data_ptr() <= p.grad.data_ptr() < f.data_ptr() + f.numel() * 4 for f in gb._flat)
    moved = [not torch.equal(p.detach(), r) for p, r in zip(params, ref_params)]
    assert all(moved) and all(bool(torch.isfinite(p).all()) for p in params)
