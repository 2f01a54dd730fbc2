"""The owner backward (l2_bwd_owner.hip) — the layer backward from the forward's saved distances
(protoseg_l2_bwd_saved / protoseg_l2_bwd_kld_saved), as the reference's autograd runs it (relu's
saved output, model.py:219) — against the oracle's autograd of model.py:203-283, and against the
recomputing backward (protoseg_l2_bwd). Tolerance: rtol 1e-4 of each gradient's own scale
(tests/test_gpu_l2.py)."""
import pytest
import torch

from oracle import kld_oracle as ko
from oracle import protoseg_oracle as po

pytestmark = pytest.mark.gpu


def _mods():
    from protoseg_amd import _lib, kld, ops
    return _lib, kld, ops


def assert_scaled_close(a, ref, rtol=1e-4, name=""):
    a, ref = a.double().cpu(), ref.double().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (a - ref).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} > {rtol:g} * scale {scale:.3e}"


def _fwd_dist(ops, x, protos, w_last, act="log", x_sigmoid=False):
    dist, _, _ = ops.prototype_layer(x, protos, w_last, 1e-4, act, True, True, False, "bf16x3", x_sigmoid)
    return dist.detach()


@pytest.mark.parametrize("B,h,w,P,K", [
    (2, 17, 17, 38, 19),     # NPT 1 (Pp 128)
    (1, 9, 11, 100, 5),      # ragged pixel tail, 5 classes
    (2, 65, 65, 190, 19),    # NPT 2: cityscapes_*_imnet.gin
    (2, 41, 41, 210, 21),    # pascal
    (4, 65, 65, 361, 19),    # NPT 3: the metric's 19 prototypes/class, tiles straddling images
    (1, 33, 35, 384, 32),    # full Pp, K = 32
    (1, 16, 16, 570, 19),    # two chunks of 285 (g_x accumulated by the second)
    (3, 7, 5, 19, 19),       # maps smaller than a tile: every tile straddles images
])
@pytest.mark.parametrize("activation", ["log", "linear"])
def test_owner_backward_vs_oracle(device, B, h, w, P, K, activation):
    _, _, ops = _mods()
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=B * 100 + h + P)
    gen = torch.Generator().manual_seed(11)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    _, _, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, None, activation)
    xd, pd, wd = x.to(device), protos.to(device), w_last.to(device)
    dist = _fwd_dist(ops, xd, pd, wd, activation)
    gx, gp, gw = ops.l2_backward(xd, pd, wd, g_logits.to(device), None, 1e-4, ops.ACT_KINDS[activation],
                                 ops.PRECISIONS["bf16x3"], True, True, True, dist)
    torch.cuda.synchronize()
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("P", [190, 361])
def test_owner_with_dense_g_dist(device, P):
    _, _, ops = _mods()
    B, h, w, K = 2, 33, 31, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=P)
    gen = torch.Generator().manual_seed(3)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = 0.01 * torch.randn(B, P, h, w, generator=gen)
    _, _, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    xd, pd, wd = x.to(device), protos.to(device), w_last.to(device)
    dist = _fwd_dist(ops, xd, pd, wd)
    gx, gp, gw = ops.l2_backward(xd, pd, wd, g_logits.to(device), g_dist.to(device), 1e-4, 0,
                                 ops.PRECISIONS["bf16x3"], True, True, True, dist)
    torch.cuda.synchronize()
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("P", [190, 361])
def test_owner_equals_recompute_within_rounding(device, P):
    """Saved distances vs recomputed ones (the one-pass / fused kernels): the same gradients to
    the split products' rounding."""
    _, _, ops = _mods()
    B, h, w, K = 4, 65, 65, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=7 + P)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(2))
    xd, pd, wd, gl = x.to(device), protos.to(device), w_last.to(device), g_logits.to(device)
    dist = _fwd_dist(ops, xd, pd, wd)
    args = (xd, pd, wd, gl, None, 1e-4, 0, ops.PRECISIONS["bf16x3"], True, True, True)
    a = ops.l2_backward(*args)
    b = ops.l2_backward(*args, dist)
    torch.cuda.synchronize()
    for u, v, name in zip(a, b, ("g_x", "g_protos", "g_w")):
        assert_scaled_close(v, u, 3e-5, name)


def test_owner_deterministic(device):
    _, _, ops = _mods()
    B, h, w, P, K = 8, 65, 65, 361, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=1)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(4))
    xd, pd, wd, gl = x.to(device), protos.to(device), w_last.to(device), g_logits.to(device)
    dist = _fwd_dist(ops, xd, pd, wd)
    args = (xd, pd, wd, gl, None, 1e-4, 0, ops.PRECISIONS["bf16x3"], True, True, True, dist)
    a = ops.l2_backward(*args)
    b = ops.l2_backward(*args)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16])
def test_owner_x_sigmoid_and_bf16_features(device, xdtype):
    _lib, _, ops = _mods()
    B, h, w, P, K = 2, 21, 23, 361, 19
    gen = torch.Generator().manual_seed(9)
    pre = (2 * torch.randn(B, 64, h, w, generator=gen)).to(xdtype)
    protos = torch.rand(P, 64, generator=gen)
    w_last = po.class_identity(P, K).t().contiguous() * 1.5 - 0.5
    g_logits = torch.randn(B, h, w, K, generator=gen)
    pre_ref = pre.float().clone().requires_grad_(True)
    protos_ref = protos.clone().requires_grad_(True)
    w_ref = w_last.clone().requires_grad_(True)
    logits, _ = po.forward_from_conv_features(torch.sigmoid(pre_ref), protos_ref[:, :, None, None], w_ref)
    logits.backward(g_logits)
    xd, pd, wd = pre.to(device), protos.to(device), w_last.to(device)
    dist = _fwd_dist(ops, xd, pd, wd, x_sigmoid=True)
    gx, gp, gw = ops.l2_backward(xd, pd, wd, g_logits.to(device), None, 1e-4, ops.ACT_KINDS["log"] | _lib.X_SIGMOID,
                                 ops.PRECISIONS["bf16x3"], True, True, True, dist)
    torch.cuda.synchronize()
    tol = 1e-4 if xdtype == torch.float32 else 1e-2
    assert_scaled_close(gx.float(), pre_ref.grad, tol, "g_pre")
    assert_scaled_close(gp, protos_ref.grad, 1e-4, "g_protos")
    assert_scaled_close(gw, w_ref.grad, 1e-4, "g_w")


@pytest.mark.parametrize("P", [190, 361, 570])
def test_owner_compact_kld_equals_dense(device, P):
    """protoseg_l2_bwd_kld_saved == protoseg_l2_bwd_saved on the expanded g_dist, bit for bit."""
    _lib, kld, ops = _mods()
    B, h, w, K = 2, 33, 35, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=P + 3)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(P + 4))
    xd, pd, wd, gl = (t.to(device) for t in (x, protos, w_last, g_logits))
    dist = _fwd_dist(ops, xd, pd, wd)
    target = ko.synthetic_targets(B, h, w, K, seed=4, block=5).to(device)
    cols, mpc = kld.prototype_columns(po.class_identity(P, K), device)
    _, _, ws = torch.ops.protoseg.kld_forward(dist, target, cols, K, mpc)
    g_loss = torch.full((), 0.25, device=device)
    g_cls, pix_cls, proto_slot = kld.kld_backward_compact(dist, target, cols, K, mpc, ws, g_loss)
    dense = ops.expand_compact((g_cls, pix_cls, proto_slot, mpc), B, P, h * w).reshape(B, P, h, w)
    prec, act = _lib.PREC_BF16X3, _lib.ACT_LOG
    ref = ops.l2_backward(xd, pd, wd, gl, dense, 1e-4, act, prec, True, True, True, dist)
    got = ops.l2_backward_kld(xd, pd, wd, gl, g_cls, pix_cls, proto_slot, mpc, 1e-4, act, prec, True, True, True, dist)
    torch.cuda.synchronize()
    for name, a, b in zip(("g_x", "g_protos", "g_w"), got, ref):
        assert torch.equal(a, b), f"{name}: max diff {(a - b).abs().max().item():.3e}"
    _, _, r_gx, r_gp, r_gw = po.forward_backward(x, protos, w_last, g_logits, dense.cpu())
    assert_scaled_close(got[0], r_gx, 1e-4, "g_x")
    assert_scaled_close(got[1], r_gp, 1e-4, "g_protos")
    assert_scaled_close(got[2], r_gw, 1e-4, "g_w")


def test_autograd_saves_distances(device, monkeypatch):
    """PPNet's autograd path hands the saved distances to the backward (owner kernel), and
    PROTOSEG_SAVE_DISTANCES=0 falls back to the recomputing backward: same gradients to rounding."""
    _, _, ops = _mods()
    seen = []
    real = ops.l2_backward

    def spy(*a, **k):
        seen.append(len(a) > 11 and a[11] is not None)
        return real(*a, **k)

    monkeypatch.setattr(ops, "l2_backward", spy)
    B, h, w, P, K = 2, 33, 35, 361, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=5)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(6)).to(device)

    def grads():
        xd = x.to(device).requires_grad_(True)
        pd = protos.to(device).requires_grad_(True)
        wd = w_last.to(device).requires_grad_(True)
        _, logits, _ = ops.prototype_layer(xd, pd, wd)
        logits.backward(g_logits)
        torch.cuda.synchronize()
        return xd.grad, pd.grad, wd.grad

    a = grads()
    monkeypatch.setattr(ops, "SAVE_DISTANCES", False)
    b = grads()
    assert seen == [True, False]
    for u, v in zip(a, b):
        assert_scaled_close(u, v, 3e-5)
