"""Oracle parity at the shapes the bench times (BASELINE configs[1] / the metric's 513x513 crop).

Smaller parity tests run B <= 2 maps, which take the forward's remainder-only schedule and the
backward's single-round loop. These run the schedules the headline measures:
  * B = 32, 65x65 (4,225 32-pixel tiles): the forward's full rounds over the resident grid plus
    its remainder round, the one-pass backward's multi-round loop with next-tile prefetch
    (P = 361) and the fused backward's (P = 190);
  * B = 8, 65x65 (1,057 tiles): the smallest batch past layout_a_grid's full-round threshold
    (l2_bf16.hip: more tiles than 3 remainder rounds over the resident grid);
  * PROTOSEG_X_SIGMOID (the add-on's nn.Sigmoid on the x load) at B = 32;
  * the compact KLD gradient (module.py:167-208) handed to the layer backward at B = 32.
Everything is checked against the oracle's torch-CPU restatement of model.py:203-283 and its
autograd, under the tolerances of tests/test_gpu_l2.py (distances 1e-4 relative with the
cancellation floor; logits and gradients 1e-4 of their own scale).
"""
import numpy as np
import pytest
import torch

from oracle import kld_oracle as ko
from oracle import protoseg_oracle as po

pytestmark = pytest.mark.gpu


def _mods():
    from protoseg_amd import _lib, kld, ops
    return _lib, kld, ops


def assert_dist_close(d, d_ref, x, protos):
    d, d_ref = d.double().cpu(), d_ref.double().cpu()
    x2 = (x.double() ** 2).sum(1, keepdim=True)
    p2 = (protos.double() ** 2).sum(1).view(1, -1, 1, 1)
    bound = 1e-4 * torch.clamp(d_ref.abs(), min=1.0) + 2e-6 * (x2 + p2)
    err = (d - d_ref).abs()
    assert bool((err <= bound).all()), f"max err {err.max().item():.3e}, worst ratio {(err / bound).max().item():.3f}"


def assert_scaled_close(a, ref, rtol=1e-4, name=""):
    a, ref = a.double().cpu(), ref.double().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (a - ref).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} > {rtol:g} * scale {scale:.3e}"


def _inputs(B, P, K=19, seed=0):
    x, protos, w_last = po.synthetic_inputs(B, 64, 65, 65, P, K, seed=seed)
    gen = torch.Generator().manual_seed(seed + 1)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, 65, 65, K, generator=gen)
    return x, protos, w_last, g_logits


@pytest.mark.parametrize("B", [32, 8])
@pytest.mark.parametrize("P", [361, 190])
def test_training_step_shape_vs_oracle(device, B, P):
    """Forward (distances, logits) and backward (g_x, g_P, g_W) at the bench's own shape, bf16x3,
    f32 feature map, through the autograd op the bench's layer step runs."""
    _, _, ops = _mods()
    x, protos, w_last, g_logits = _inputs(B, P, seed=B * 1000 + P)
    xd = x.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd, precision="bf16x3")
    logits.backward(g_logits.to(device))
    torch.cuda.synchronize()
    r_logits, r_dist, r_gx, r_gp, r_gw = po.forward_backward(x, protos, w_last, g_logits, None)
    assert_dist_close(dist.detach(), r_dist, x, protos)
    assert_scaled_close(logits.detach(), r_logits, 1e-4, "logits")
    assert_scaled_close(xd.grad, r_gx, 1e-4, "g_x")
    assert_scaled_close(pd.grad, r_gp, 1e-4, "g_protos")
    assert_scaled_close(wd.grad, r_gw, 1e-4, "g_w")


@pytest.mark.parametrize("P", [361, 190])
def test_x_sigmoid_at_bench_shape(device, P):
    """PROTOSEG_X_SIGMOID at B = 32: the layer reads the add-on's pre-activation and applies the
    sigmoid on load; the oracle runs torch.sigmoid then the restated layer, gradient w.r.t. the
    pre-activation."""
    _, _, ops = _mods()
    B, K = 32, 19
    gen = torch.Generator().manual_seed(P)
    pre = 2.0 * torch.randn(B, 64, 65, 65, generator=gen)
    protos = torch.rand(P, 64, generator=gen)
    w_last = po.last_layer_init(po.class_identity(P, K)) + 0.05 * torch.randn(K, P, generator=gen)
    g_logits = torch.randn(B, 65, 65, K, generator=gen)
    xd = pre.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd, precision="bf16x3", x_sigmoid=True)
    logits.backward(g_logits.to(device))
    torch.cuda.synchronize()
    pre_ref = pre.clone().requires_grad_(True)
    p_ref = protos.clone().requires_grad_(True)
    w_ref = w_last.clone().requires_grad_(True)
    sx = torch.sigmoid(pre_ref)
    r_logits, r_dist = po.forward_from_conv_features(sx, p_ref[:, :, None, None], w_ref)
    r_logits.backward(g_logits)
    assert_dist_close(dist.detach(), r_dist.detach(), sx.detach(), protos)
    assert_scaled_close(logits.detach(), r_logits.detach(), 1e-4, "logits")
    assert_scaled_close(xd.grad, pre_ref.grad, 1e-4, "g_pre")
    assert_scaled_close(pd.grad, p_ref.grad, 1e-4, "g_protos")
    assert_scaled_close(wd.grad, w_ref.grad, 1e-4, "g_w")


def test_compact_kld_backward_at_bench_shape(device):
    """The KLD step's backward at B = 32, P = 361: (1) the KLD distance gradient (dense kernel)
    against the oracle's float64 closed form of module.py:167-208; (2) the layer backward with the
    compact gradient equals the one with the dense g_dist bit for bit; (3) that backward against
    the oracle's autograd with the same g_dist."""
    _lib, kld, ops = _mods()
    B, P, K = 32, 361, 19
    x, protos, w_last, g_logits = _inputs(B, P, seed=77)
    xd, pd, wd, gl = (t.to(device) for t in (x, protos, w_last, g_logits))
    dist = ops.prototype_layer(xd, pd, wd)[0]
    target = ko.synthetic_targets(B, 65, 65, K, seed=5, block=9).to(device)
    ident = po.class_identity(P, K)
    cols, mpc = kld.prototype_columns(ident, device)
    loss, npairs, ws = torch.ops.protoseg.kld_forward(dist, target, cols, K, mpc)
    g_loss = torch.full((), 0.25, device=device)
    dense = torch.ops.protoseg.kld_backward(dist, target, cols, K, mpc, ws, g_loss)
    g_cls, pix_cls, proto_slot = kld.kld_backward_compact(dist, target, cols, K, mpc, ws, g_loss)
    torch.cuda.synchronize()
    # (1) the KLD loss and gradient on the kernel's own distances
    ref_loss, ref_n, ref_g = ko.kld_loss_float64(dist.cpu().numpy(), target.cpu().numpy(), cols.cpu().numpy(), K)
    assert int(npairs) == ref_n and ref_n > 0
    assert abs(float(loss) - ref_loss) <= 1e-5
    ref_g = torch.from_numpy(0.25 * ref_g)
    assert_scaled_close(dense, ref_g, 1e-4, "kld g_dist")
    assert torch.equal(dense.cpu() == 0, ref_g == 0)
    # (2) compact == dense through the layer backward
    assert _lib.load().protoseg_l2_bwd_kld_supported(B, 64, 65, 65, P, K, _lib.F32, _lib.PREC_BF16X3, mpc) == 1
    prec, act = _lib.PREC_BF16X3, _lib.ACT_LOG
    ref = ops.l2_backward(xd, pd, wd, gl, dense, 1e-4, act, prec, True, True, True)
    got = ops.l2_backward_kld(xd, pd, wd, gl, g_cls, pix_cls, proto_slot, mpc, 1e-4, act, prec, True, True, True)
    torch.cuda.synchronize()
    for name, a, b in zip(("g_x", "g_protos", "g_w"), got, ref):
        assert torch.equal(a, b), f"{name}: max diff {(a - b).abs().max().item():.3e}"
    # (3) the layer backward with that g_dist against the oracle's autograd
    _, _, r_gx, r_gp, r_gw = po.forward_backward(x, protos, w_last, g_logits, dense.cpu())
    assert_scaled_close(got[0], r_gx, 1e-4, "g_x")
    assert_scaled_close(got[1], r_gp, 1e-4, "g_protos")
    assert_scaled_close(got[2], r_gw, 1e-4, "g_w")


def test_forward_full_round_boundary(device):
    """Batches either side of layout_a_grid's full-round threshold (3 remainder rounds over the
    resident grid, l2_bf16.hip): every distance, logit row and tile edge lands where the oracle
    puts it (ragged 33x47 maps make tiles straddle images)."""
    _, _, ops = _mods()
    P, K = 361, 19
    for B in (15, 16, 17):
        x, protos, w_last = po.synthetic_inputs(B, 64, 33, 47, P, K, seed=B)
        dist, logits, _ = ops.prototype_layer(x.to(device), protos.to(device), w_last.to(device))
        torch.cuda.synchronize()
        r_logits, r_dist = po.forward_from_conv_features(x, protos[:, :, None, None], w_last)
        assert_dist_close(dist, r_dist, x, protos)
        assert_scaled_close(logits, r_logits, 1e-4, f"logits B={B}")
        assert np.isfinite(dist.cpu().numpy()).all()
