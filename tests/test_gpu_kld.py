"""Parity of the HIP KLD loss (module.py:167-208) and its gradient with the oracle.

Tolerances: loss within 1e-5 absolute (it is a mean of exp(-kld) in [0, 1]); the pair count
exactly; the distance gradient within 1e-4 of its own scale (f32 softmax / KL sums in a
different order than torch's). Zero gradient off each prototype's class pixels, exactly.
"""
import os

import numpy as np
import pytest
import torch

from oracle import kld_oracle as ko
from oracle import protoseg_oracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

pytestmark = pytest.mark.gpu


def _kld():
    from protoseg_amd import kld
    return kld


def _run(dist, target, ident, device, g_loss=1.0):
    kld = _kld()
    d = dist.to(device).requires_grad_(True)
    loss = kld.kld_loss(d, target.to(device), ident)
    (loss * g_loss).backward()
    torch.cuda.synchronize()
    return float(loss), d.grad.detach().cpu()


def _check(dist, target, ident, device, g_loss=1.0):
    loss, grad = _run(dist, target, ident, device, g_loss)
    ref_loss, ref_n, ref_grad = ko.kld_loss_and_grad(dist, target.long(), ident, g_loss)
    assert abs(loss - ref_loss) <= 1e-5, (loss, ref_loss, ref_n)
    scale = ref_grad.abs().max().item()
    err = (grad - ref_grad).abs().max().item()
    assert err <= 1e-4 * scale + 1e-12, f"grad err {err:.3e} scale {scale:.3e}"
    assert torch.equal(grad == 0, ref_grad == 0) or scale == 0.0
    return loss, ref_n


def test_kld_matches_golden(device):
    kld = _kld()
    g = np.load(os.path.join(GOLDEN, "kld_small.npz"))
    K = int(g["num_classes"])
    pc = torch.from_numpy(g["proto_class"]).to(device)
    d = torch.from_numpy(g["dist"]).to(device)
    t = torch.from_numpy(g["target"]).to(device)
    loss, npairs, ws = torch.ops.protoseg.kld_forward(d, t, pc, K, 2)
    g_dist = torch.ops.protoseg.kld_backward(d, t, pc, K, 2, ws, torch.ones((), device=device))
    torch.cuda.synchronize()
    assert int(npairs) == int(g["n_pairs"])
    assert abs(float(loss) - float(g["loss"])) <= 1e-5
    ref = torch.from_numpy(g["g_dist"])
    assert (g_dist.cpu() - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
    assert kld.MAX_PER_CLASS == 32


@pytest.mark.parametrize("ldtype", [torch.int64, torch.int32, torch.uint8])
@pytest.mark.parametrize("B,h,w,P,K,block", [
    (2, 9, 11, 38, 19, 3),      # 2 prototypes per class
    (2, 17, 19, 190, 19, 4),    # cityscapes: 10 per class
    (1, 20, 23, 361, 19, 5),    # 19 per class
    (1, 12, 13, 90, 3, 2),      # 30 per class (DenseNet config), 3 classes
    (3, 5, 7, 10, 5, 1),        # pixel-level labels, many tiny classes
])
def test_kld_vs_oracle(device, ldtype, B, h, w, P, K, block):
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed=B * 7 + P)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1))
    target = ko.synthetic_targets(B, h, w, K, seed=h * w, block=block).to(ldtype)
    ident = po.class_identity(P, K)
    loss, n = _check(dist, target, ident, device, g_loss=0.25)
    assert n > 0 and 0.0 < loss <= 1.0


@pytest.mark.parametrize("B,h,w,P,K,block", [
    (1, 65, 65, 361, 19, 8),    # 5 pixel ranges (<= 8: the merge's register path), 19 per class
                                # (the partial / compact kernels' recomputed-exp form)
    (1, 97, 97, 38, 19, 6),     # 10 ranges: the merge's general path
    (1, 129, 67, 190, 19, 8),   # 9 ranges at 10 per class (stored-exp form)
])
def test_kld_vs_oracle_many_ranges(device, B, h, w, P, K, block):
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed=h + P)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1))
    target = ko.synthetic_targets(B, h, w, K, seed=w, block=block)
    ident = po.class_identity(P, K)
    loss, n = _check(dist, target, ident, device, g_loss=0.5)
    assert n > 0 and 0.0 < loss <= 1.0


def test_kld_no_pairs_and_skip_rules(device):
    P, K, h, w = 6, 3, 4, 4
    dist = torch.rand(1, P, h, w)
    ident = po.class_identity(P, K)
    only_k = torch.full((1, h * w), K)
    loss, grad = _run(dist, only_k, ident, device)
    assert loss == 0.0 and grad.abs().max().item() == 0.0
    single = torch.full((1, h * w), K)
    single[0, 3] = 1
    loss, grad = _run(dist, single, ident, device)
    assert loss == 0.0 and grad.abs().max().item() == 0.0
    void = torch.zeros(1, h * w, dtype=torch.long)   # void pairs with class-0 prototypes
    _check(dist, void, ident, device)


def test_kld_known_answer_identical_prototypes(device):
    h = w = 9
    dist = torch.rand(2, 1, h, w).repeat(1, 6, 1, 1)
    ident = po.class_identity(6, 3)
    target = ko.synthetic_targets(2, h, w, 2, seed=3, block=3)
    loss, grad = _run(dist, target, ident, device)
    assert abs(loss - 1.0) < 1e-6
    assert grad.abs().max().item() < 1e-6


def test_kld_full_crop_properties(device):
    """BASELINE shape (B=4, 65x65, P=190): loss in (0, 1], gradient zero off each prototype's
    class pixels, and a finite-difference check of the loss along the gradient direction."""
    kld = _kld()
    B, h, w, P, K = 4, 65, 65, 190, 19
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed=5)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1)).to(device)
    target = ko.synthetic_targets(B, h, w, K, seed=6, block=8).to(device)
    ident = po.class_identity(P, K)
    d = dist.clone().requires_grad_(True)
    loss = kld.kld_loss(d, target, ident)
    loss.backward()
    g = d.grad
    assert 0.0 < float(loss) <= 1.0
    cls = (torch.arange(P, device=device) // 10).view(1, P, 1)
    off_class = (target.view(B, 1, -1) != cls).view(B, P, h, w)
    assert g[off_class].abs().max().item() == 0.0
    step = 1e-2 / g.norm()
    up = float(kld.kld_loss(dist + step * g, target, ident))
    dn = float(kld.kld_loss(dist - step * g, target, ident))
    fd = (up - dn) / 2.0
    assert abs(fd - float(step * g.norm() ** 2)) <= 0.05 * abs(fd) + 1e-7
    ref_loss, _ = ko.kld_loss(dist[:1].cpu(), target[:1].cpu(), ident)
    one = float(kld.kld_loss(dist[:1], target[:1], ident))
    assert abs(one - float(ref_loss)) <= 1e-5


def test_kld_deterministic(device):
    kld = _kld()
    x, protos, _ = po.synthetic_inputs(2, 64, 30, 31, 190, 19, seed=8)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(190, 64, 1, 1)).to(device)
    target = ko.synthetic_targets(2, 30, 31, 19, seed=9, block=4).to(device)
    ident = po.class_identity(190, 19)
    outs = []
    for _ in range(2):
        d = dist.clone().requires_grad_(True)
        loss = kld.kld_loss(d, target, ident)
        loss.backward()
        outs.append((loss.detach().clone(), d.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
