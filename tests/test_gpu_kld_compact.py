"""The KLD gradient in its compact layout (module.py:167-208 autograd, no [B, P, H, W] tensor).

protoseg_kld_backward_compact stores d loss / d dist only at the prototypes of each pixel's own
class; protoseg_l2_bwd_kld expands it inside the layer backward's owners. Both must reproduce the
dense path bit for bit: the compact kernel runs the dense kernel's operation sequence per pixel,
and the layer kernels add the same f32 value to the same accumulator, so the tests use
torch.equal. The dense path itself is held to the oracle by test_gpu_kld.py / test_gpu_l2.py.
"""
import os

import pytest
import torch

from oracle import kld_oracle as ko
from oracle import protoseg_oracle as po

pytestmark = pytest.mark.gpu


def _mods():
    from protoseg_amd import _lib, kld, ops
    return _lib, kld, ops


@pytest.mark.parametrize("B,h,w,P,K,block", [
    (2, 9, 11, 38, 19, 3),
    (2, 17, 19, 190, 19, 4),
    (1, 20, 23, 361, 19, 5),
    (3, 5, 7, 10, 5, 1),
    (2, 65, 65, 190, 19, 8),
])
def test_compact_expands_to_dense(device, B, h, w, P, K, block):
    _lib, kld, ops = _mods()
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed=B * 5 + P)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1)).to(device)
    target = ko.synthetic_targets(B, h, w, K, seed=h + w, block=block).to(device)
    ident = po.class_identity(P, K)
    cols, mpc = kld.prototype_columns(ident, device)
    loss, npairs, ws = torch.ops.protoseg.kld_forward(dist, target, cols, K, mpc)
    g_loss = torch.full((), 0.25, device=device)
    dense = torch.ops.protoseg.kld_backward(dist, target, cols, K, mpc, ws, g_loss)
    g_cls, pix_cls, proto_slot = kld.kld_backward_compact(dist, target, cols, K, mpc, ws, g_loss)
    expanded = ops.expand_compact((g_cls, pix_cls, proto_slot, mpc), B, P, h * w).reshape(B, P, h, w)
    torch.cuda.synchronize()
    assert torch.equal(expanded, dense)
    # slots: the class column and the rank among that class's prototypes (ascending id)
    slot = proto_slot.cpu()
    col = cols.cpu()
    for p in range(P):
        assert int(slot[p]) >> 8 == int(col[p])
        assert int(slot[p]) & 255 == int((col[:p] == col[p]).sum())
    # pixel classes: the label where its (image, class) group adds pairs, else -1
    t = target.reshape(B, -1).long().cpu()
    pc = pix_cls.reshape(B, -1).cpu().long()
    assert bool(((pc == t) | (pc == -1)).all())
    ref_loss, ref_n, _ = ko.kld_loss_and_grad(dist.cpu(), target.long().cpu(), ident, 0.25)
    assert abs(float(loss) - ref_loss) <= 1e-5 and int(npairs) == ref_n


def _layer_inputs(B, h, w, P, K, seed):
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=seed)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(seed + 1))
    return x, protos, w_last, g_logits


@pytest.mark.parametrize("P,bwd", [(190, "fused"), (570, "fused"), (38, "fused"), (38, "wave"), (190, "wave"),
                                   (361, "wave"), (570, "wave")])
def test_l2_bwd_kld_equals_dense(device, bwd_kernel, P, bwd):
    """protoseg_l2_bwd_kld == protoseg_l2_bwd on the expanded g_dist, bit for bit, for the fused
    (P <= 192 per chunk) and wave-owned (P <= 384 per chunk) kernels, chunked P included."""
    _lib, kld, ops = _mods()
    bwd_kernel(bwd)
    B, h, w, K = 2, 33, 35, 19
    x, protos, w_last, g_logits = _layer_inputs(B, h, w, P, K, seed=P + 3)
    xd, pd, wd, gl = (t.to(device) for t in (x, protos, w_last, g_logits))
    dist = ops.prototype_layer(xd, pd, wd)[0]
    target = ko.synthetic_targets(B, h, w, K, seed=4, block=5).to(device)
    cols, mpc = kld.prototype_columns(po.class_identity(P, K), device)
    _, _, ws = torch.ops.protoseg.kld_forward(dist, target, cols, K, mpc)
    g_loss = torch.full((), 0.25, device=device)
    g_cls, pix_cls, proto_slot = kld.kld_backward_compact(dist, target, cols, K, mpc, ws, g_loss)
    dense = ops.expand_compact((g_cls, pix_cls, proto_slot, mpc), B, P, h * w).reshape(B, P, h, w)
    assert _lib.load().protoseg_l2_bwd_kld_supported(B, 64, h, w, P, K, _lib.F32, _lib.PREC_BF16X3, mpc) == 1
    prec, act = _lib.PREC_BF16X3, _lib.ACT_LOG
    ref = ops.l2_backward(xd, pd, wd, gl, dense, 1e-4, act, prec, True, True, True)
    got = ops.l2_backward_kld(xd, pd, wd, gl, g_cls, pix_cls, proto_slot, mpc, 1e-4, act, prec, True, True, True)
    torch.cuda.synchronize()
    for name, a, b in zip(("g_x", "g_protos", "g_w"), got, ref):
        assert torch.equal(a, b), f"{name}: max diff {(a - b).abs().max().item():.3e}"


def test_l2_bwd_kld_refuses_unserved_shapes(device):
    _lib, _, _ = _mods()
    lib = _lib.load()
    assert lib.protoseg_l2_bwd_kld_supported(2, 64, 9, 9, 190, 19, _lib.BF16, _lib.PREC_BF16X3, 10) == 0
    assert lib.protoseg_l2_bwd_kld_supported(2, 64, 9, 9, 190, 19, _lib.F32, _lib.PREC_F32, 10) == 0
    assert lib.protoseg_l2_bwd_kld_supported(2, 128, 9, 9, 190, 19, _lib.F32, _lib.PREC_BF16X3, 10) == 0


def _train_grads(device, P, extra_dist_loss, dense_only, x_sigmoid=False):
    """Gradients of CE-like + 0.25 * KLD (+ an optional second use of the distances)."""
    _lib, kld, ops = _mods()
    B, h, w, K = 2, 33, 35, 19
    x, protos, w_last, g_logits = _layer_inputs(B, h, w, P, K, seed=11)
    xd = x.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    target = ko.synthetic_targets(B, h, w, K, seed=12, block=5).to(device)
    ident = po.class_identity(P, K)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd, x_sigmoid=x_sigmoid)
    d_in = dist * 1.0 if dense_only else dist  # a new tensor carries no hand-off: the dense path
    loss = (logits * g_logits.to(device)).sum() + 0.25 * kld.kld_loss(d_in, target, ident)
    if extra_dist_loss:
        loss = loss + (dist * torch.linspace(0, 1e-3, dist.numel(), device=device).view_as(dist)).sum()
    loss.backward()
    torch.cuda.synchronize()
    return [t.grad.detach().clone() for t in (xd, pd, wd)]


@pytest.mark.parametrize("P", [190, 361])
@pytest.mark.parametrize("extra", [False, True])
def test_autograd_hands_off_compact_gradient(device, monkeypatch, P, extra):
    """kld_loss on PPNet's distances: the layer receives the compact gradient (counted here),
    with the gradients of the dense path bit for bit; a second consumer of the distances adds its
    dense gradient (the deposit is then expanded into it)."""
    _lib, kld, ops = _mods()
    calls = {"compact": 0, "l2_kld": 0}
    real_compact, real_l2 = kld.kld_backward_compact, ops.l2_backward_kld

    def count_compact(*a, **k):
        calls["compact"] += 1
        return real_compact(*a, **k)

    def count_l2(*a, **k):
        calls["l2_kld"] += 1
        return real_l2(*a, **k)

    monkeypatch.setattr(kld, "kld_backward_compact", count_compact)
    monkeypatch.setattr(ops, "l2_backward_kld", count_l2)
    got = _train_grads(device, P, extra, dense_only=False)
    assert calls["compact"] == 1
    assert calls["l2_kld"] == (0 if extra else 1)
    ref = _train_grads(device, P, extra, dense_only=True)
    assert calls["compact"] == 1  # the reference run took the dense path
    for name, a, b in zip(("g_x", "g_protos", "g_w"), got, ref):
        if extra:  # dense + expanded deposit summed in a different order than autograd's
            assert (a - b).abs().max().item() <= 1e-6 * max(1.0, b.abs().max().item()), name
        else:
            assert torch.equal(a, b), f"{name}: max diff {(a - b).abs().max().item():.3e}"


def test_autograd_hand_off_with_fused_sigmoid(device):
    got = _train_grads(device, 190, False, dense_only=False, x_sigmoid=True)
    ref = _train_grads(device, 190, False, dense_only=True, x_sigmoid=True)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def _layer_and_kld(device, P, K, seed=21):
    _lib, kld, ops = _mods()
    B, h, w = 2, 33, 35
    x, protos, w_last, g_logits = _layer_inputs(B, h, w, P, K, seed=seed)
    xd = x.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    target = ko.synthetic_targets(B, h, w, K, seed=seed + 1, block=5).to(device)
    ident = po.class_identity(P, K)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd)
    return (xd, pd, wd), dist, logits, g_logits.to(device), target, ident


def _dense_kld_grad(dist, target, ident, g_loss=0.25):
    _, kld, _ = _mods()
    cols, mpc = kld.prototype_columns(ident, dist.device)
    K = ident.shape[1]
    _, _, ws = torch.ops.protoseg.kld_forward(dist.detach(), target, cols, K, mpc)
    return torch.ops.protoseg.kld_backward(dist.detach(), target, cols, K, mpc, ws,
                                           torch.full((), g_loss, device=dist.device))


def test_wide_family_takes_the_dense_kld_gradient(device):
    """K = 40 classes at C = 64 runs the layer on the wide family, which reads a dense g_dist only:
    protoseg_l2_bwd_kld_supported refuses, so kld_loss hands autograd the dense gradient and the
    layer's gradients equal the dense-only path's (the compact gradient was dropped)."""
    _lib, kld, ops = _mods()
    P, K = 80, 40
    assert _lib.load().protoseg_l2_bwd_kld_supported(2, 64, 33, 35, P, K, _lib.F32, _lib.PREC_BF16X3, 2) == 0

    def grads(dense_only):
        leaves, dist, logits, gl, target, ident = _layer_and_kld(device, P, K)
        d_in = dist * 1.0 if dense_only else dist
        loss = (logits * gl).sum() + 0.25 * kld.kld_loss(d_in, target, ident)
        loss.backward()
        torch.cuda.synchronize()
        return [t.grad.clone() for t in leaves]

    got, ref = grads(False), grads(True)
    for name, a, b in zip(("g_x", "g_protos", "g_w"), got, ref):
        assert torch.equal(a, b), name
    assert ref[1].abs().max().item() > 0


def test_hand_off_autograd_grad_on_distances(device):
    """autograd.grad(kld, distances) never runs the layer backward: the KLD node returns the dense
    gradient (not the hand-off's zero) and leaves no deposit behind."""
    _, kld, _ = _mods()
    _, dist, _, _, target, ident = _layer_and_kld(device, 190, 19)
    loss = 0.25 * kld.kld_loss(dist, target, ident)
    (g,) = torch.autograd.grad(loss, dist)
    torch.cuda.synchronize()
    assert torch.equal(g, _dense_kld_grad(dist, target, ident))
    assert dist._protoseg_sink.deposits == []


def test_hand_off_retain_grad_and_hooks_see_real_values(device):
    _, kld, _ = _mods()
    leaves, dist, logits, gl, target, ident = _layer_and_kld(device, 190, 19)
    dist.retain_grad()
    seen = []
    dist.register_hook(lambda g: seen.append(g.clone()))
    loss = 0.25 * kld.kld_loss(dist, target, ident) + (logits * gl).sum()
    loss.backward()
    torch.cuda.synchronize()
    dense = _dense_kld_grad(dist, target, ident)
    assert torch.equal(dist.grad, dense) and torch.equal(seen[0], dense)
    leaves2, dist2, logits2, gl2, target2, ident2 = _layer_and_kld(device, 190, 19)
    loss2 = 0.25 * kld.kld_loss(dist2 * 1.0, target2, ident2) + (logits2 * gl2).sum()
    loss2.backward()
    for a, b in zip(leaves, leaves2):
        assert torch.equal(a.grad, b.grad)


def test_hand_off_retain_graph_and_partial_passes(device):
    """A retain_graph replay sums each pass's gradient once, and a pass that stops at the distances
    (backward(inputs=[dist])) leaves no deposit for the next full pass."""
    _, kld, _ = _mods()
    leaves, dist, logits, gl, target, ident = _layer_and_kld(device, 361, 19)
    loss = 0.25 * kld.kld_loss(dist, target, ident) + (logits * gl).sum()
    loss.backward(inputs=[dist], retain_graph=True)
    assert torch.equal(dist.grad, _dense_kld_grad(dist, target, ident))
    loss.backward(retain_graph=True)
    first = [t.grad.clone() for t in leaves]
    loss.backward()
    torch.cuda.synchronize()
    leaves2, dist2, logits2, gl2, target2, ident2 = _layer_and_kld(device, 361, 19)
    loss2 = 0.25 * kld.kld_loss(dist2 * 1.0, target2, ident2) + (logits2 * gl2).sum()
    loss2.backward()
    for a, b, f in zip(leaves, leaves2, first):
        assert torch.equal(f, b.grad)
        assert torch.equal(a.grad, b.grad + b.grad)


def test_hand_off_explicit_inputs_with_the_layer_behind(device):
    """a pass with explicit inputs that captures the distances AND runs the layer's
    backward (backward(inputs=[dist, protos]); autograd.grad over [dist, a non-leaf upstream of x])
    must see the dense KLD gradient at the distances, and the layer's gradients must equal the
    dense path's: the hand-off is only taken in plain backward() passes."""
    _, kld, ops = _mods()
    P, K = 190, 19

    def run(mode, dense_only):
        leaves, dist, logits, gl, target, ident = _layer_and_kld(device, P, K)
        d_in = dist * 1.0 if dense_only else dist
        loss = 0.25 * kld.kld_loss(d_in, target, ident) + (logits * gl).sum()
        if mode == "inputs":
            loss.backward(inputs=[dist, leaves[1]])
            out = [dist.grad, leaves[1].grad]
        else:
            out = list(torch.autograd.grad(loss, [dist, leaves[1], leaves[2]]))
        torch.cuda.synchronize()
        return [t.detach().clone() for t in out], dist, target, ident

    for mode in ("inputs", "grad"):
        got, dist, target, ident = run(mode, False)
        ref, _, _, _ = run(mode, True)
        assert torch.equal(got[0], _dense_kld_grad(dist, target, ident)), mode
        for a, b in zip(got, ref):
            assert torch.equal(a, b), mode
        assert dist._protoseg_sink.deposits == []

    # autograd.grad over the distances and a non-leaf tensor upstream of x
    _lib, kld, ops = _mods()
    B, h, w = 2, 33, 35
    x, protos, w_last, g_logits = _layer_inputs(B, h, w, P, K, seed=31)
    target = ko.synthetic_targets(B, h, w, K, seed=32, block=5).to(device)
    ident = po.class_identity(P, K)

    def grads(dense_only):
        x0 = x.to(device).requires_grad_(True)
        feats = x0 * 1.0  # a non-leaf before the layer's x
        dist, logits, _ = ops.prototype_layer(feats, protos.to(device), w_last.to(device))
        d_in = dist * 1.0 if dense_only else dist
        loss = 0.25 * kld.kld_loss(d_in, target, ident) + (logits * g_logits.to(device)).sum()
        gd, gf = torch.autograd.grad(loss, [dist, feats])
        torch.cuda.synchronize()
        return gd, gf, dist

    gd, gf, dist = grads(False)
    rd, rf, _ = grads(True)
    assert torch.equal(gd, _dense_kld_grad(dist, target, ident)) and torch.equal(gd, rd)
    assert torch.equal(gf, rf)


def test_kld_gradient_ignores_stale_workspace(device):
    """The KLD workspace comes from torch's caching allocator uninitialised. The merge kernel never
    writes KL's diagonal; a NaN left there by an earlier tensor once reached the gradient through
    w_ii * KL_ii = 0 * NaN (found when this file ran after the B = 32 parity tests)."""
    _lib, kld, ops = _mods()
    junk = [torch.full((n,), float("nan"), device=device) for n in (1 << 12, 1 << 16, 1 << 20, 1 << 23)]
    del junk
    B, h, w, P, K = 2, 9, 11, 38, 19
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed=B * 5 + P)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1)).to(device)
    target = ko.synthetic_targets(B, h, w, K, seed=h + w, block=3).to(device)
    ident = po.class_identity(P, K)
    cols, mpc = kld.prototype_columns(ident, device)
    _, _, ws = torch.ops.protoseg.kld_forward(dist, target, cols, K, mpc)
    g_loss = torch.full((), 0.25, device=device)
    dense = torch.ops.protoseg.kld_backward(dist, target, cols, K, mpc, ws, g_loss)
    g_cls, pix_cls, proto_slot = kld.kld_backward_compact(dist, target, cols, K, mpc, ws, g_loss)
    expanded = ops.expand_compact((g_cls, pix_cls, proto_slot, mpc), B, P, h * w).reshape(B, P, h, w)
    torch.cuda.synchronize()
    assert not bool(torch.isnan(dense).any()) and not bool(torch.isnan(expanded).any())
    assert torch.equal(expanded, dense)
    _, _, ref = ko.kld_loss_and_grad(dist.cpu(), target.long().cpu(), ident, 0.25)
    assert (dense.cpu() - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
