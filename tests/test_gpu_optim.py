"""protoseg_amd.optim.Adam (protoseg_adam_step, adam.hip) against torch.optim.Adam, the
reference's optimizer (segmentation/module.py:391). Bar: parameters within 1e-6 relative (+1e-7
absolute) of torch's after several steps (same f32 arithmetic up to the order of the bias
correction's division); a HIP-graph capture of step() replays as successive steps."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(device, shapes, seed):
    gen = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.rand(s, generator=gen).to(device)) for s in shapes]


def _grads(ps, step, seed):
    gen = torch.Generator().manual_seed(seed * 1000 + step)
    for p in ps:
        p.grad = torch.randn(p.shape, generator=gen).to(p.device)


@pytest.mark.parametrize("wd", [0.0, 5e-4])
def test_adam_matches_torch(device, wd):
    from protoseg_amd.optim import Adam
    shapes = [(361, 64, 1, 1), (19, 361), (7,), (1,)] + [(33, 5)] * 7  # 11 tensors: 2 launches
    ours = _params(device, shapes, 1)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    groups = lambda ps: [{"params": ps[:2], "lr": 2.5e-4}, {"params": ps[2:], "lr": 1e-3,  # noqa: E731
                                                            "weight_decay": wd}]
    opt = Adam(groups(ours), weight_decay=wd)
    opt_ref = torch.optim.Adam(groups(ref), weight_decay=wd, foreach=False)
    for step in range(6):
        _grads(ours, step, 2)
        for a, b in zip(ref, ours):
            a.grad = b.grad.clone()
        opt.step()
        opt_ref.step()
    for a, b in zip(ours, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max().item()


def test_adam_graph_replay_is_successive_steps(device):
    from protoseg_amd.optim import Adam
    ours = _params(device, [(190, 64), (19, 190)], 3)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt, opt_ref = Adam(ours, lr=2.5e-4), torch.optim.Adam(ref, lr=2.5e-4, foreach=False)
    _grads(ours, 0, 4)
    for a, b in zip(ref, ours):
        a.grad = b.grad.clone()
    opt.step()  # first step eager (state allocation), then three graph replays
    opt_ref.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        opt.step()
    torch.cuda.current_stream().wait_stream(s)
    # capture does not run the update; replays do, each one step further
    for _ in range(3):
        g.replay()
        opt_ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max().item()


def test_adam_rejects_non_f32(device):
    from protoseg_amd import _lib
    from protoseg_amd.optim import Adam
    p = torch.nn.Parameter(torch.zeros(4, device=device, dtype=torch.float64))
    p.grad = torch.ones_like(p)
    with pytest.raises(_lib.ProtosegError):
        Adam([p]).step()


def test_adam_state_dict_round_trip_with_torch(device):
    """Checkpoint resume both ways: torch.optim.Adam -> ours -> torch, the bias correction
    continuing from the saved per-parameter step (the step is in state_dict)."""
    from protoseg_amd.optim import Adam
    ours = _params(device, [(361, 64), (19, 361)], 5)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt_ref = torch.optim.Adam(ref, lr=2.5e-4, weight_decay=5e-4, foreach=False)
    for step in range(3):
        _grads(ref, step, 6)
        opt_ref.step()
    with torch.no_grad():
        for a, b in zip(ours, ref):
            a.copy_(b)
    opt = Adam(ours, lr=2.5e-4, weight_decay=5e-4)
    opt.load_state_dict(copy.deepcopy(opt_ref.state_dict()))  # a checkpoint: no shared tensors
    for step in range(3, 5):
        _grads(ours, step, 6)
        for a, b in zip(ref, ours):
            a.grad = b.grad.clone()
        opt.step()
        opt_ref.step()
    for a, b in zip(ours, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max().item()
    sd = opt.state_dict()
    assert [float(s["step"]) for s in sd["state"].values()] == [5.0, 5.0]
    # and back into torch
    ref2 = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt_ref2 = torch.optim.Adam(ref2, lr=2.5e-4, weight_decay=5e-4, foreach=False)
    opt_ref2.load_state_dict(copy.deepcopy(sd))
    _grads(ours, 9, 6)
    for a, b in zip(ref2, ours):
        a.grad = b.grad.clone()
    opt.step()
    opt_ref2.step()
    for a, b in zip(ours, ref2):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (a - b).abs().max().item()


def test_adam_per_parameter_step_counts(device):
    """A parameter without a gradient on some steps keeps its own step count (torch semantics),
    and an empty tensor still advances its count."""
    from protoseg_amd.optim import Adam
    ours = _params(device, [(40,), (33, 5)], 8) + [torch.nn.Parameter(torch.zeros(0, device=device))]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt, opt_ref = Adam(ours, lr=1e-3), torch.optim.Adam(ref, lr=1e-3, foreach=False)
    for step in range(5):
        _grads(ours, step, 9)
        if step % 2 == 1:
            ours[1].grad = None  # skipped on odd steps
        for a, b in zip(ref, ours):
            a.grad = None if b.grad is None else b.grad.clone()
        opt.step()
        opt_ref.step()
    for a, b in zip(ours, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)
    steps = [float(s["step"]) for s in opt.state_dict()["state"].values()]
    assert steps == [float(s["step"]) for s in opt_ref.state_dict()["state"].values()] == [5.0, 3.0, 5.0]
