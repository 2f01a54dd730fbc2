"""Parity of the HIP prototype layer (forward + backward) with the oracle, through the C ABI.

Tolerances (north_star: "fp32 distances within 1e-4 rel"): distances are compared as
|d - d_ref| <= 1e-4 * max(|d_ref|, 1) + 2e-6 * (||x||^2 + ||p||^2); the second term is the
cancellation bound of the expanded form relu(||x||^2 - 2x.p + ||p||^2) that both the reference
and the kernel evaluate in f32 (it matters only where d << ||x||^2). Activations, logits and
gradients: rtol 1e-4 of the tensor's own scale.
"""
import os

import numpy as np
import pytest
import torch

from oracle import protoseg_oracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

pytestmark = pytest.mark.gpu


def _ops():
    from protoseg_amd import ops
    return ops


def _norm_bound(x, protos):
    x2 = (x.double() ** 2).sum(1, keepdim=True)  # [B,1,h,w]
    p2 = (protos.double() ** 2).sum(1).view(1, -1, 1, 1)
    return x2 + p2


def assert_dist_close(d, d_ref, x, protos):
    d, d_ref = d.double().cpu(), d_ref.double().cpu()
    bound = 1e-4 * torch.clamp(d_ref.abs(), min=1.0) + 2e-6 * _norm_bound(x.cpu(), protos.cpu())
    err = (d - d_ref).abs()
    assert bool((err <= bound).all()), f"max err {err.max().item():.3e}, worst ratio {(err / bound).max().item():.3f}"


def assert_scaled_close(a, ref, rtol=1e-4, name=""):
    a, ref = a.double().cpu(), ref.double().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (a - ref).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} > {rtol:g} * scale {scale:.3e}"


PRECISIONS = ["bf16x3", "bf16x6", "f32"]


def prec(name):
    return _ops().PRECISIONS[name]


def run_layer(x, protos, w_last, activation="log", with_act=False, device="cuda:0", precision="bf16x3"):
    ops = _ops()
    return ops.prototype_layer(x.to(device), protos.to(device), w_last.to(device), 1e-4, activation,
                               True, True, with_act, precision)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", ["l2_small", "l2_ragged"])
def test_forward_matches_golden(device, name, precision):
    g = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    x, protos, w_last = (torch.from_numpy(g[k]) for k in ("x", "protos", "w_last"))
    dist, logits, act = run_layer(x, protos, w_last, with_act=True, device=device, precision=precision)
    torch.cuda.synchronize()
    assert_dist_close(dist, torch.from_numpy(g["dist"]), x, protos)
    assert_scaled_close(logits, torch.from_numpy(g["logits"]), 1e-4, "logits")
    assert_scaled_close(act, torch.from_numpy(g["act"]), 1e-4, "act")


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("name", ["l2_small", "l2_ragged"])
def test_backward_matches_golden(device, name, precision):
    ops = _ops()
    g = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    x, protos, w_last, g_logits, g_dist = (torch.from_numpy(g[k]).to(device) for k in
                                           ("x", "protos", "w_last", "g_logits", "g_dist"))
    gx, gp, gw = ops.l2_backward(x, protos, w_last, g_logits, None, 1e-4, 0, prec(precision), True, True, True)
    torch.cuda.synchronize()
    assert_scaled_close(gx, torch.from_numpy(g["g_x"]), 1e-4, "g_x")
    assert_scaled_close(gp, torch.from_numpy(g["g_protos"]), 1e-4, "g_protos")
    assert_scaled_close(gw, torch.from_numpy(g["g_w"]), 1e-4, "g_w")
    gx2, gp2, _ = ops.l2_backward(x, protos, w_last, g_logits, g_dist, 1e-4, 0, prec(precision), True, True, False)
    assert_scaled_close(gx2, torch.from_numpy(g["g_x_with_gdist"]), 1e-4, "g_x(+g_dist)")
    assert_scaled_close(gp2, torch.from_numpy(g["g_protos_with_gdist"]), 1e-4, "g_protos(+g_dist)")


@pytest.mark.parametrize("B,C,h,w,P,K", [
    (1, 64, 1, 1, 19, 19),        # a single pixel
    (2, 64, 5, 3, 32, 19),        # P exactly one tile
    (1, 64, 33, 1, 33, 5),        # P one over a tile, pixel tail of 1
    (2, 32, 9, 9, 10, 2),         # C = 32
    (1, 128, 6, 7, 64, 32),       # C = 128, K = 32 (max)
    (2, 64, 65, 65, 190, 19),     # cityscapes crop, 10 prototypes/class
    (1, 64, 65, 65, 361, 19),     # 19 prototypes/class
    (2, 64, 41, 41, 210, 21),     # pascal_*.gin: 21 classes x 10, 321x321 window -> 41x41
    (2, 64, 21, 21, 50, 5),       # cells.gin: 5 classes x 10, MSC scale 0.5 of the 321 window
])
@pytest.mark.parametrize("activation", ["log", "linear"])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_forward_backward_vs_oracle(device, B, C, h, w, P, K, activation, precision):
    x, protos, w_last = po.synthetic_inputs(B, C, h, w, P, K, seed=B * 1000 + C + h + P)
    gen = torch.Generator().manual_seed(5)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    dist, logits, _ = run_layer(x, protos, w_last, activation, device=device, precision=precision)
    ref_logits, ref_dist, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, None, activation)
    assert_dist_close(dist, ref_dist, x, protos)
    assert_scaled_close(logits, ref_logits, 1e-4, "logits")
    ops = _ops()
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device), g_logits.to(device), None,
                                 1e-4, ops.ACT_KINDS[activation], prec(precision), True, True, True)
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("hw", [32, 65])
@pytest.mark.parametrize("K", [2, 3])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_config0_mds_new_layer_shapes(device, K, hw, precision):
    """BASELINE configs[0] (mds_new.gin:6-7: prototype_shape (30, 64, 1, 1), num_classes 3, batch 2;
    BASELINE names 2 classes, so K = 2 too) at its 256x256 (32x32 map) and 513x513 (65x65 map)
    crops: forward and backward against the oracle, with an upstream g_dist (the KLD-style path)."""
    B, C, P = 2, 64, 30
    x, protos, w_last = po.synthetic_inputs(B, C, hw, hw, P, K, seed=30 + K + hw)
    gen = torch.Generator().manual_seed(K * 100 + hw)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, hw, hw, K, generator=gen)
    g_dist = torch.randn(B, P, hw, hw, generator=gen) * 0.05
    dist, logits, act = run_layer(x, protos, w_last, with_act=True, device=device, precision=precision)
    ref_logits, ref_dist, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    assert_dist_close(dist, ref_dist, x, protos)
    assert_scaled_close(logits, ref_logits, 1e-4, "logits")
    ref_act = po.distance_2_similarity(ref_dist.permute(0, 2, 3, 1).reshape(-1, P))
    assert_scaled_close(act.reshape(-1, P), ref_act, 1e-4, "act")
    ops = _ops()
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device), g_logits.to(device),
                                 g_dist.to(device), 1e-4, 0, prec(precision), True, True, True)
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("P", [57, 361])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_bf16_features(device, precision, P):
    """bf16 feature maps are read exactly (bf16 -> f32 is exact) and computed in f32 (P = 361:
    the backward runs over prototype chunks, g_x accumulated in bf16 — tolerance 1e-2 holds)."""
    x, protos, w_last = po.synthetic_inputs(2, 64, 17, 19, P, 19, seed=3)
    xb = x.to(torch.bfloat16)
    dist, logits, _ = run_layer(xb, protos, w_last, device=device, precision=precision)
    ref_logits, ref_dist = po.forward_from_conv_features(xb.float(), protos[:, :, None, None], w_last)
    assert_dist_close(dist, ref_dist, xb.float(), protos)
    assert_scaled_close(logits, ref_logits, 1e-4, "logits")
    ops = _ops()
    g_logits = torch.randn(2, 17, 19, 19)
    gx, gp, _ = ops.l2_backward(xb.to(device), protos.to(device), w_last.to(device), g_logits.to(device), None,
                                1e-4, 0, prec(precision), True, True, False)
    assert gx.dtype == torch.bfloat16
    _, _, ref_gx, ref_gp, _ = po.forward_backward(xb.float(), protos, w_last, g_logits, None)
    assert_scaled_close(gx.float(), ref_gx, 1e-2, "g_x(bf16 out)")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")


@pytest.mark.parametrize("precision", PRECISIONS)
def test_known_answer_zero_distance(device, precision):
    """x equal to a prototype at a pixel -> d = 0 (relu clamps) -> act = log(1/1e-4) = 9.2103."""
    x, protos, w_last = po.synthetic_inputs(1, 64, 4, 4, 19, 19, seed=11)
    x[0, :, 2, 3] = protos[7]
    dist, logits, act = run_layer(x, protos, w_last, with_act=True, device=device, precision=precision)
    d = dist[0, 7, 2, 3].item()
    assert d <= 2e-6 * 2 * (protos[7] ** 2).sum().item()
    a = act.view(1, 4, 4, 19)[0, 2, 3, 7].item()
    assert abs(a - float(np.log((d + 1) / (d + 1e-4)))) < 1e-4
    if d == 0.0:
        assert abs(a - 9.210340371976184) < 1e-5


@pytest.mark.parametrize("precision", PRECISIONS)
def test_distances_match_float64_bruteforce(device, precision):
    """Size-independent property at the full 65x65 crop: d == ||x - p||^2 within the f32 bound."""
    x, protos, w_last = po.synthetic_inputs(4, 64, 65, 65, 190, 19, seed=17)
    dist, _, _ = run_layer(x, protos, w_last, device=device, precision=precision)
    xd = x.double().permute(0, 2, 3, 1).reshape(-1, 64)
    exact = torch.cdist(xd, protos.double()) ** 2
    exact = exact.reshape(4, 65, 65, 190).permute(0, 3, 1, 2)
    assert_dist_close(dist, exact, x, protos)


@pytest.mark.parametrize("precision", PRECISIONS)
def test_deterministic(device, precision):
    """No atomics on the float path: two runs are bitwise identical."""
    ops = _ops()
    x, protos, w_last = po.synthetic_inputs(3, 64, 40, 41, 190, 19, seed=23)
    x, protos, w_last = x.to(device), protos.to(device), w_last.to(device)
    g = torch.randn(3, 40, 41, 19, device=device)
    r1 = ops.l2_backward(x, protos, w_last, g, None, 1e-4, 0, prec(precision), True, True, True)
    r2 = ops.l2_backward(x, protos, w_last, g, None, 1e-4, 0, prec(precision), True, True, True)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


def test_ppnet_autograd_matches_oracle(device):
    """PPNet.forward_from_conv_features + autograd through the custom op == oracle autograd."""
    from protoseg_amd.model import PPNet
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    feats = deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[])
    net = PPNet(feats, 513, (38, 64, 1, 1), None, 19, add_on_layers_type="deeplab_simple",
                patch_classification=True).to(device)
    x, _, _ = po.synthetic_inputs(2, 64, 9, 9, 38, 19, seed=29)
    xd = x.to(device).requires_grad_(True)
    logits, dist = net.forward_from_conv_features(xd)
    loss = logits.square().sum() + 0.1 * dist.sum()
    loss.backward()
    ref_logits, ref_dist = po.forward_from_conv_features(x, net.prototype_vectors.detach().cpu(),
                                                         net.last_layer.weight.detach().cpu())
    g_logits = 2 * ref_logits
    _, _, ref_gx, ref_gp, ref_gw = po.forward_backward(x, net.prototype_vectors.detach().cpu(),
                                                       net.last_layer.weight.detach().cpu(), g_logits,
                                                       torch.full_like(ref_dist, 0.1))
    assert_scaled_close(logits.detach(), ref_logits, 1e-4, "logits")
    assert_scaled_close(xd.grad, ref_gx, 1e-4, "g_x")
    assert_scaled_close(net.prototype_vectors.grad.reshape(38, 64), ref_gp, 1e-4, "g_protos")
    assert_scaled_close(net.last_layer.weight.grad, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("activation", ["log", "linear"])
def test_gradient_through_return_activations(device, activation):
    """model.py:280-281: forward_from_conv_features(..., return_activations=True) returns
    (logits, activations); a loss on both back-propagates as the reference's autograd does."""
    from protoseg_amd.model import PPNet
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    feats = deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[])
    net = PPNet(feats, 513, (38, 64, 1, 1), None, 19, add_on_layers_type="deeplab_simple",
                prototype_activation_function=activation, patch_classification=True).to(device)
    x, _, _ = po.synthetic_inputs(2, 64, 9, 10, 38, 19, seed=31)
    coef = torch.randn(2 * 9 * 10, 38, generator=torch.Generator().manual_seed(4))
    xd = x.to(device).requires_grad_(True)
    logits, acts = net.forward_from_conv_features(xd, return_activations=True)
    (logits.square().sum() + (acts * coef.to(device)).sum()).backward()
    xr = x.clone().requires_grad_(True)
    pr = net.prototype_vectors.detach().cpu().clone().requires_grad_(True)
    wr = net.last_layer.weight.detach().cpu().clone().requires_grad_(True)
    rl, ra = po.forward_from_conv_features(xr, pr, wr, activation, return_activations=True)
    (rl.square().sum() + (ra * coef).sum()).backward()
    assert_scaled_close(acts.detach(), ra.detach(), 1e-4, "acts")
    assert_scaled_close(xd.grad, xr.grad, 1e-4, "g_x")
    assert_scaled_close(net.prototype_vectors.grad, pr.grad, 1e-4, "g_protos")
    assert_scaled_close(net.last_layer.weight.grad, wr.grad, 1e-4, "g_w")


def test_cpu_tensors_fail_loudly():
    from protoseg_amd import ops
    x, protos, w_last = po.synthetic_inputs(1, 64, 2, 2, 19, 19)
    with pytest.raises((RuntimeError, NotImplementedError)):
        ops.prototype_layer(x, protos, w_last)


def test_timing_events_bracket_one_kernel():
    """protoseg_timing_events (bench.py's roofline timer) brackets the named kernel only: its
    interval is positive, no longer than the whole call's, and it is silent once cleared."""
    import ctypes

    from protoseg_amd import _lib

    dev = torch.device("cuda:0")
    x, protos, w_last = po.synthetic_inputs(8, 64, 33, 33, 190, 19, seed=5)
    x, protos, w_last = x.to(dev), protos.to(dev), w_last.to(dev)
    dist = torch.empty(8, 190, 33, 33, device=dev)
    logits = torch.empty(8, 33, 33, 19, device=dev)
    lib = _lib.load()
    stream = _lib.stream_of(dev)
    null = ctypes.c_void_p(None)

    def fwd():
        _lib.call("protoseg_l2_fwd", _lib.ptr(x), _lib.F32, 8, 64, 33, 33, _lib.ptr(protos), 190, _lib.ptr(w_last), 19,
                  1e-4, _lib.ACT_LOG, _lib.PREC_BF16X3, _lib.ptr(dist), null, _lib.ptr(logits), stream)

    fwd()
    k0, k1, c0, c1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    for e in (k0, k1):
        e.record()
    torch.cuda.synchronize()
    assert lib.protoseg_timing_events(b"l2_fwd_bf16_kernel", ctypes.c_void_p(k0.cuda_event),
                                      ctypes.c_void_p(k1.cuda_event)) == 0
    try:
        c0.record()
        fwd()
        c1.record()
        torch.cuda.synchronize()
    finally:
        assert lib.protoseg_timing_events(None, None, None) == 0
    kern, call = k0.elapsed_time(k1), c0.elapsed_time(c1)
    assert 0.0 < kern <= call, (kern, call)
    assert lib.protoseg_timing_kernel() == b"l2_fwd_bf16_kernel"
    fwd()  # cleared: the kernel events keep their last interval
    torch.cuda.synchronize()
    assert k0.elapsed_time(k1) == kern


def test_timing_events_family_prefix_reports_the_family_that_ran():
    """bench.py times kernels by family prefix and the hook names the kernel that ran: the
    forward in f32 precision runs the f32 family; the P = 361 x-backward runs the bf16 family
    over prototype chunks (the hook keeps the last chunk's launch)."""
    import ctypes

    from protoseg_amd import _lib

    dev = torch.device("cuda:0")
    B, h, w, P, K = 2, 17, 17, 361, 19
    x, protos, w_last = (t.to(dev) for t in po.synthetic_inputs(B, 64, h, w, P, K, seed=6))
    g_logits = torch.randn(B, h, w, K, device=dev)
    g_x = torch.empty_like(x)
    lib = _lib.load()
    null = ctypes.c_void_p(None)
    k0, k1 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
    for e in (k0, k1):
        e.record()
    torch.cuda.synchronize()
    for family, expect_bf16 in (("l2_fwd", False), ("l2_bwd_x", True)):
        assert lib.protoseg_timing_events(family.encode(), ctypes.c_void_p(k0.cuda_event),
                                          ctypes.c_void_p(k1.cuda_event)) == 0
        try:
            if family == "l2_fwd":
                dist = torch.empty(B, P, h, w, device=dev)
                _lib.call("protoseg_l2_fwd", _lib.ptr(x), _lib.F32, B, 64, h, w, _lib.ptr(protos), P, _lib.ptr(w_last),
                          K, 1e-4, _lib.ACT_LOG, _lib.PREC_F32, _lib.ptr(dist), null, null, _lib.stream_of(dev))
            else:
                _lib.call("protoseg_l2_bwd", _lib.ptr(x), _lib.F32, B, 64, h, w, _lib.ptr(protos), P, _lib.ptr(w_last),
                          K, 1e-4, _lib.ACT_LOG, _lib.PREC_BF16X3, _lib.ptr(g_logits), null, _lib.ptr(g_x), null, null,
                          null, 0, _lib.stream_of(dev))
            torch.cuda.synchronize()
        finally:
            assert lib.protoseg_timing_events(None, None, None) == 0
        name = lib.protoseg_timing_kernel().decode()
        assert name == (f"{family}_bf16_kernel" if expect_bf16 else f"{family}_kernel"), name
        assert k0.elapsed_time(k1) > 0.0


@pytest.mark.parametrize("with_logits", [True, False])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_prototype_chunked_backward_with_g_dist(device, precision, with_logits):
    """P = 361 backward with an upstream distance gradient (the KLD path, module.py:167-208):
    the bf16 family runs over prototype chunks reading g_dist rows at (b * P + p0 + p)."""
    B, h, w, P, K = 2, 23, 29, 361, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=361)
    gen = torch.Generator().manual_seed(8)
    g_logits = torch.randn(B, h, w, K, generator=gen) if with_logits else None
    g_dist = torch.randn(B, P, h, w, generator=gen) * 0.1
    _, _, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    ops = _ops()
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device),
                                 g_logits.to(device) if with_logits else None, g_dist.to(device), 1e-4, 0,
                                 prec(precision), True, True, with_logits)
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x(+g_dist, chunked)")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos(+g_dist, chunked)")
    if with_logits:
        assert_scaled_close(gw, ref_gw, 1e-4, "g_w(chunked)")



@pytest.mark.parametrize("activation", ["log", "linear"])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_prototype_chunked_forward_backward_p570(device, precision, activation):
    """30 prototypes/class (P = 570, the DenseNet config's prototype count): the forward runs in
    two prototype chunks (distance / activation rows at b * P + p0 + p, logits summed), the
    backward in three; all outputs against the oracle, g_dist included."""
    B, h, w, P, K = 2, 16, 16, 570, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=570)
    gen = torch.Generator().manual_seed(9)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = torch.randn(B, P, h, w, generator=gen) * 0.1
    dist, logits, act = run_layer(x, protos, w_last, activation, with_act=True, device=device, precision=precision)
    ref_logits, ref_dist, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist, activation)
    assert_dist_close(dist, ref_dist, x, protos)
    assert_scaled_close(logits, ref_logits, 1e-4, "logits")
    ref_act = po.distance_2_similarity(ref_dist.permute(0, 2, 3, 1).reshape(-1, P), activation)
    assert_scaled_close(act.reshape(-1, P), ref_act, 1e-4, "act")
    ops = _ops()
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device), g_logits.to(device),
                                 g_dist.to(device), 1e-4, ops.ACT_KINDS[activation], prec(precision), True, True, True)
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("C,P,K", [(128, 400, 19), (32, 1200, 5)])
def test_f32_family_prototype_chunks_other_widths(device, C, P, K):
    """The f32 family (any C of the family) over prototype chunks: C = 128 stages at most 224
    prototypes per launch, C = 32 a few hundred; forward and backward against the oracle."""
    B, h, w = 1, 7, 9
    x, protos, w_last = po.synthetic_inputs(B, C, h, w, P, K, seed=C + P)
    gen = torch.Generator().manual_seed(P)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = torch.randn(B, P, h, w, generator=gen) * 0.1
    dist, logits, _ = run_layer(x, protos, w_last, device=device, precision="f32")
    ref_logits, ref_dist, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    assert_dist_close(dist, ref_dist, x, protos)
    assert_scaled_close(logits, ref_logits, 1e-4, "logits")
    ops = _ops()
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device), g_logits.to(device),
                                 g_dist.to(device), 1e-4, 0, prec("f32"), True, True, True)
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


def test_fp16_features_widen_exactly(device):
    """fp16 feature maps (DenseNet fp16 config): computed as their exact f32 widening; g_x comes
    back in fp16 through autograd."""
    ops = _ops()
    x, protos, w_last = po.synthetic_inputs(2, 64, 16, 16, 570, 19, seed=16)
    xh = x.half()
    xd = xh.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, protos.to(device), w_last.to(device))
    g_logits = torch.randn(2, 16, 16, 19, generator=torch.Generator().manual_seed(3))
    logits.backward(g_logits.to(device))
    ref_logits, ref_dist, ref_gx, _, _ = po.forward_backward(xh.float(), protos, w_last, g_logits, None)
    assert_dist_close(dist, ref_dist, xh.float(), protos)
    assert_scaled_close(logits.detach(), ref_logits, 1e-4, "logits")
    assert xd.grad.dtype == torch.float16
    assert_scaled_close(xd.grad.float(), ref_gx, 2e-3, "g_x(fp16)")


def _pre_activation(B, C, h, w, seed, dtype=torch.float32):
    """The deeplab_simple add-on's input (§8d: X = sigmoid(N(0, 2^2)), so pre = N(0, 2^2))."""
    return (2.0 * torch.randn(B, C, h, w, generator=torch.Generator().manual_seed(seed))).to(dtype)


@pytest.mark.parametrize("P,xdtype,with_gdist", [(38, torch.float32, False), (190, torch.float32, True),
                                                 (190, torch.bfloat16, False), (361, torch.float32, True),
                                                 (570, torch.float32, False)])
def test_x_sigmoid_fused_on_load_vs_oracle(device, P, xdtype, with_gdist):
    """PROTOSEG_X_SIGMOID (model.py:124-128's nn.Sigmoid applied on the layer's x load): forward
    and backward equal the oracle on sigmoid(pre); g_x is the pre-activation's gradient
    g_x * s (1 - s). P = 361 / 570 run the prototype chunks (g_x accumulated across chunks)."""
    ops = _ops()
    B, C, h, w, K = 2, 64, 23, 29, 19
    pre = _pre_activation(B, C, h, w, seed=P, dtype=xdtype)
    _, protos, w_last = po.synthetic_inputs(B, C, h, w, P, K, seed=P + 1)
    gen = torch.Generator().manual_seed(P + 2)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = 0.05 * torch.randn(B, P, h, w, generator=gen) if with_gdist else None
    assert ops.x_sigmoid_supported(pre.to(device), P, K, "bf16x3")
    prd = pre.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(prd, pd, wd, 1e-4, "log", precision="bf16x3", x_sigmoid=True)
    outs, grads = [logits], [g_logits.to(device)]
    if with_gdist:
        outs.append(dist)
        grads.append(g_dist.to(device))
    torch.autograd.backward(outs, grads)
    s = torch.sigmoid(pre.float())
    ref_logits, ref_dist, ref_gx, ref_gp, ref_gw = po.forward_backward(s, protos, w_last, g_logits, g_dist)
    assert_dist_close(dist.detach(), ref_dist, s, protos)
    assert_scaled_close(logits.detach(), ref_logits, 1e-4, "logits")
    rtol = 1e-4 if xdtype == torch.float32 else 1e-2  # bf16 g_x output
    assert prd.grad.dtype == xdtype
    assert_scaled_close(prd.grad.float(), ref_gx * s * (1 - s), rtol, "g_pre")
    assert_scaled_close(pd.grad, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(wd.grad, ref_gw, 1e-4, "g_w")


def test_x_sigmoid_other_precisions_take_torch_sigmoid(device):
    """bf16x6 / f32 have no on-load sigmoid: prototype_layer applies torch.sigmoid first (same
    result), and the C ABI refuses the flag for them (fails loudly, no silent misuse)."""
    from protoseg_amd import _lib
    ops = _ops()
    pre = _pre_activation(1, 64, 9, 11, seed=3)
    _, protos, w_last = po.synthetic_inputs(1, 64, 9, 11, 38, 19, seed=4)
    for precision in ("bf16x6", "f32"):
        assert not ops.x_sigmoid_supported(pre, 38, 19, precision)
        d, lg, _ = ops.prototype_layer(pre.to(device), protos.to(device), w_last.to(device), precision=precision,
                                       x_sigmoid=True)
        ref_logits, ref_dist = po.forward_from_conv_features(torch.sigmoid(pre), protos[:, :, None, None], w_last)
        assert_dist_close(d, ref_dist, torch.sigmoid(pre), protos)
        assert_scaled_close(lg, ref_logits, 1e-4, "logits")
        with pytest.raises(_lib.ProtosegError, match="X_SIGMOID"):
            ops.l2_forward(pre.to(device), protos.to(device), w_last.to(device), 1e-4, _lib.X_SIGMOID,
                           ops.PRECISIONS[precision], True, True, False)


def test_ppnet_forward_image_fuses_add_on_sigmoid(device):
    """PPNet.forward(image) (model.py:239-246): the add-on's sigmoid runs inside the layer kernels
    (the backbone output goes in as the pre-activation); logits / distances and every gradient
    (prototypes, last layer, backbone through g_pre) equal the oracle on sigmoid(features(image))."""
    from protoseg_amd.model import PPNet
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    torch.manual_seed(0)
    feats = deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[])
    net = PPNet(feats, 513, (190, 64, 1, 1), None, 19, add_on_layers_type="deeplab_simple",
                patch_classification=True).to(device)
    net.eval()
    assert net._sigmoid_free_add_on() is not None
    image = torch.randn(2, 3, 65, 65, generator=torch.Generator().manual_seed(8)).to(device)
    logits, dist = net(image)
    (logits.square().sum() + 0.1 * dist.sum()).backward()
    g_head = [p.grad.detach().clone() for p in net.features.parameters() if p.grad is not None]
    assert g_head, "backbone gets a gradient through the fused sigmoid"
    with torch.no_grad():
        pre = net.features(image).float().cpu()
    s = torch.sigmoid(pre)
    protos = net.prototype_vectors.detach().cpu()
    wl = net.last_layer.weight.detach().cpu()
    ref_logits, ref_dist = po.forward_from_conv_features(s, protos, wl)
    assert_dist_close(dist.detach(), ref_dist, s, protos.reshape(190, 64))
    assert_scaled_close(logits.detach(), ref_logits, 1e-4, "logits")
    _, _, _, ref_gp, ref_gw = po.forward_backward(s, protos, wl, 2 * ref_logits, torch.full_like(ref_dist, 0.1))
    assert_scaled_close(net.prototype_vectors.grad.reshape(190, 64), ref_gp, 1e-4, "g_protos")
    assert_scaled_close(net.last_layer.weight.grad, ref_gw, 1e-4, "g_w")
    # the unfused path (sigmoid materialised by nn.Sigmoid) gives the same backbone gradient
    net.zero_grad()
    net.fuse_add_on_sigmoid = False
    l2, d2 = net(image)
    (l2.square().sum() + 0.1 * d2.sum()).backward()
    g_ref = [p.grad for p in net.features.parameters() if p.grad is not None]
    for a, b in zip(g_head, g_ref):
        assert_scaled_close(a, b, 1e-3, "backbone grad")


@pytest.mark.parametrize("kh,kw,C", [(3, 3, 64), (2, 3, 32)])
def test_kxk_prototypes_vs_oracle(device, kh, kw, C):
    """k x k prototypes (model.py:203-221 with prototype_shape[2:] > 1): the layer runs on the
    unfolded map (wide family at C k k); distances, logits and every gradient against the oracle's
    F.conv2d formulation and its autograd."""
    ops = _ops()
    B, h, w, P, K = 2, 13, 17, 38, 19
    gen = torch.Generator().manual_seed(kh * 10 + kw)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen))
    protos = torch.rand(P, C, kh, kw, generator=gen)
    w_last = po.last_layer_init(po.class_identity(P, K))
    g_logits = torch.randn(B, h - kh + 1, w - kw + 1, K, generator=gen)
    xr, pr, wr = (t.clone().requires_grad_(True) for t in (x, protos, w_last))
    ref_logits, ref_dist = po.forward_from_conv_features(xr, pr, wr)
    (ref_logits * g_logits).sum().backward()
    xd, pd, wd = (t.to(device).requires_grad_(True) for t in (x, protos, w_last))
    dist, logits, _ = ops.prototype_layer(xd, pd, wd)
    (logits * g_logits.to(device)).sum().backward()
    torch.cuda.synchronize()
    assert dist.shape == (B, P, h - kh + 1, w - kw + 1)
    xu = torch.nn.functional.unfold(x, (kh, kw)).reshape(B, C * kh * kw, h - kh + 1, w - kw + 1)
    assert_dist_close(dist, ref_dist.detach(), xu, protos.reshape(P, -1))
    assert_scaled_close(logits, ref_logits.detach(), 1e-4, "logits")
    assert_scaled_close(xd.grad, xr.grad, 1e-4, "g_x")
    assert_scaled_close(pd.grad, pr.grad, 1e-4, "g_protos")
    assert_scaled_close(wd.grad, wr.grad, 1e-4, "g_w")
