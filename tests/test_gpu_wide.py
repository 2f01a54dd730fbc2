"""The wide family (l2_wide.hip): any prototype depth C and any class count K.

The reference's own construct_PPNet default is prototype_shape = (2000, 512, 1, 1) with 200
classes (model.py:394); the C in {32, 64, 128}, K <= 32 kernels do not hold it. These tests run
that shape (and C = 256, odd depths, K > 32 at C = 64) through PPNet's layer op and the push
argmin, against the oracle (model.py:203-283 restated op for op, autograd for the backward;
push.py:195-263 restated). Products are bf16x3 splits for the default BF16X3 requests (fp16 maps:
the fp16 distance GEMM with two-term prototypes) and exact f32 for F32 requests: distances within
1e-4 relative (+ a floor of 1e-6 (||x||^2 + ||p||^2) for the expanded form's cancellation),
logits and gradients within 1e-4 of their own scale (f32 sums over C / P / pixels in a different
order than torch-CPU's).
"""
import numpy as np
import pytest
import torch

from oracle import protoseg_oracle as po
from oracle import push_oracle as pu

pytestmark = pytest.mark.gpu


def _close(got, ref, name, rel=1e-4):
    got = got.detach().double().cpu()
    ref = ref.double()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    assert err <= rel * max(scale, 1e-30), f"{name}: max err {err:.3e} (scale {scale:.3e})"


def _inputs(B, C, h, w, P, K, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.sigmoid(2.0 * torch.randn(B, C, h, w, generator=gen))
    protos = torch.rand(P, C, generator=gen)
    ident = torch.zeros(P, K)
    for p in range(P):
        ident[p, p % K] = 1  # every class holds prototypes even when P is not a multiple of K
    w_last = po.last_layer_init(ident)
    g_logits = torch.randn(B, h, w, K, generator=gen) / (B * h * w)
    g_dist = torch.randn(B, P, h, w, generator=gen) * 1e-3
    return x, protos, w_last, g_logits, g_dist


@pytest.mark.parametrize("B,C,h,w,P,K", [
    (1, 512, 7, 9, 2000, 200),   # construct_PPNet's default (model.py:394)
    (2, 256, 9, 11, 2000, 200),
    (2, 48, 13, 7, 190, 19),     # a depth outside {32, 64, 128}
    (2, 64, 9, 10, 120, 40),     # more than 32 classes at C = 64
    (1, 96, 5, 6, 4500, 19),     # P beyond the chunked families' 4096
])
def test_wide_layer_forward_backward_vs_oracle(device, B, C, h, w, P, K):
    from protoseg_amd import _lib, ops
    assert _lib.load().protoseg_l2_supported(C, P, K) == 1
    x, protos, w_last, g_logits, g_dist = _inputs(B, C, h, w, P, K, seed=C + P + K)
    xd = x.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd)
    torch.autograd.backward([logits, dist], [g_logits.to(device), g_dist.to(device)])
    torch.cuda.synchronize()
    r_logits, r_dist, r_gx, r_gp, r_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    floor = 1e-6 * ((x ** 2).sum(1).max() + (protos ** 2).sum(1).max()).item()
    derr = (dist.detach().cpu() - r_dist).abs()
    assert bool((derr <= 1e-4 * r_dist.abs() + floor).all()), f"distances: max err {derr.max().item():.3e}"
    _close(logits, r_logits, "logits")
    _close(xd.grad, r_gx, "g_x")
    _close(pd.grad, r_gp, "g_protos")
    _close(wd.grad, r_gw, "g_w")


@pytest.mark.parametrize("B,C,h,w,P,K,dt", [
    (2, 192, 8, 8, 100, 7, torch.float32),     # g_x on 192-row tiles (pre_mi 3), every tile full
    (2, 320, 8, 8, 130, 7, torch.float16),     # 192-row tiles, the last one partial (rows 320..383)
    (1, 1000, 8, 4, 70, 5, torch.bfloat16),    # 256-row tiles (pre_mi 4), the last one partial
    (3, 256, 16, 16, 600, 19, torch.float16),  # g_P split over the pixels, several row tiles
])
def test_wide_pre_split_backward_vs_oracle(device, B, C, h, w, P, K, dt):
    """The pre-split backward (launch_bwd_wide_pre: G_s split in its GEMM's epilogue, g_x and g_P
    on wide_pre_gemm_kernel, HW a multiple of 32) across its tile choices and feature-map dtypes,
    against the oracle on the same (rounded) feature map: gradients within 1e-4 of their scale
    (bf16x3 products), g_x within its storage dtype's rounding."""
    from protoseg_amd import ops
    x, protos, w_last, g_logits, g_dist = _inputs(B, C, h, w, P, K, seed=C + P)
    xr = x.to(dt)
    xd = xr.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd)
    torch.autograd.backward([logits, dist], [g_logits.to(device), g_dist.to(device)])
    torch.cuda.synchronize()
    r_logits, r_dist, r_gx, r_gp, r_gw = po.forward_backward(xr.float(), protos, w_last, g_logits, g_dist)
    _close(logits, r_logits, "logits")
    _close(xd.grad.float(), r_gx, "g_x", rel=1e-4 if dt == torch.float32 else 1e-2)
    _close(pd.grad, r_gp, "g_protos")
    _close(wd.grad, r_gw, "g_w")


def test_wide_layer_bf16_x_and_activations(device):
    """bf16 feature maps (widened exactly), the activation output and the linear activation."""
    from protoseg_amd import ops
    B, C, h, w, P, K = 2, 160, 6, 7, 300, 37
    x, protos, w_last, g_logits, _ = _inputs(B, C, h, w, P, K, seed=3)
    xb = x.to(torch.bfloat16)
    xd = xb.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    _, logits, acts = ops.prototype_layer(xd, pd, wd, with_dist=False, with_act=True)
    logits.backward(g_logits.to(device))
    r_logits, r_act = po.forward_from_conv_features(xb.float(), protos, w_last, return_activations=True)
    _close(logits, r_logits, "logits")
    _close(acts, r_act, "activations")
    _, _, r_gx, r_gp, r_gw = po.forward_backward(xb.float(), protos, w_last, g_logits, None)
    _close(xd.grad.float(), r_gx, "g_x (bf16)", rel=1e-2)  # g_x is stored in bf16
    _close(pd.grad, r_gp, "g_protos")
    _close(wd.grad, r_gw, "g_w")
    dist_lin, logits_lin, _ = ops.prototype_layer(xd.detach(), pd.detach(), wd.detach(), activation="linear")
    r_ll, r_dl = po.forward_from_conv_features(xb.float(), protos, w_last, activation="linear")
    _close(logits_lin, r_ll, "logits (linear)")


def _bitmask_words(labels, h, w, words):
    """Multi-plane class bitmask [words, h*w] from the reference's class -> patch sets."""
    sets = pu.class_to_patch_index_dict(labels, h, w, 32 * words)
    out = np.zeros((words, h * w), dtype=np.uint32)
    for k, patches in sets.items():
        for (i, j) in patches:
            out[k >> 5, i * w + j] |= np.uint32(1 << (k & 31))
    return out


@pytest.mark.parametrize("C,P,K", [(256, 2000, 200), (512, 400, 200), (48, 190, 19), (64, 190, 19)])
def test_wide_push_argmin_vs_oracle(device, C, P, K):
    """push.py:195-263 at >32 classes / wide depths: class planes bit-exact, minima and (where
    separated) patch indices equal to the oracle's, runner-ups, and push_distances reproducing
    exactly the distances the argmin saw (the exact-tie resolution's premise)."""
    from protoseg_amd import push
    n, h, w, H, W = 2, 9, 11, 40, 47
    words = push.mask_words(K)
    rng = np.random.default_rng(C + K)
    labels = rng.integers(0, K + 1, size=(n, H, W)).astype(np.int64)
    x, protos, _, _, _ = _inputs(n, C, h, w, P, K, seed=P)
    pcls = (torch.arange(P) % K).to(torch.int32)
    mask = push.patch_class_mask(torch.from_numpy(labels).to(device), h, w, words=words)
    mk = mask.cpu().numpy().view(np.uint32)
    if words == 1:
        mk = mk[None]
    for i in range(n):
        assert np.array_equal(mk[:, i], _bitmask_words(labels[i], h, w, words))
    xd, pd, pcd = x.to(device), protos.to(device), pcls.to(device)
    keys, second = push.push_argmin(xd, pd, pcd, mask, with_second=True)
    d, patch, found = push.decode_keys(keys.cpu())
    ds, _, fs = push.decode_keys(second.cpu())
    r_dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, C, 1, 1))
    exact = 0
    for i in range(n):
        sets = pu.class_to_patch_index_dict(labels[i], h, w, K)
        dm = r_dist[i].reshape(P, -1).numpy()
        dk = push.push_distances(xd[i], pd, words).cpu().numpy()  # the argmin's own arithmetic
        for p in range(0, P, max(1, P // 97)):
            cand = sorted(pi * w + pj for pi, pj in sets[int(pcls[p])])
            assert bool(found[i, p]) == (len(cand) > 0)
            if not cand:
                continue
            ref = dm[p, cand]
            assert abs(float(d[i, p]) - ref.min()) <= 1e-4 * ref.min() + 1e-4
            own = dk[p, cand]
            assert float(d[i, p]) == own.min() and int(patch[i, p]) == cand[int(np.argmin(own))]
            if len(cand) > 1:
                assert bool(fs[i, p]) and float(ds[i, p]) == np.sort(own)[1]
            srt = np.sort(ref)
            if len(cand) == 1 or srt[1] - srt[0] > 1e-5 * (1 + srt[0]) + 1e-4:
                assert int(patch[i, p]) == cand[int(np.argmin(ref))]
                exact += 1
    assert exact > 0


def test_ppnet_default_shape_constructs(device):
    """construct_PPNet's reference default (prototype_shape (2000, 512, 1, 1), 200 classes) runs
    a forward + backward on the HIP path."""
    from protoseg_amd import ops
    x, protos, w_last, g_logits, _ = _inputs(1, 512, 4, 5, 2000, 200, seed=9)
    xd = x.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, protos.to(device), w_last.to(device))
    logits.backward(g_logits.to(device))
    torch.cuda.synchronize()
    assert dist.shape == (1, 2000, 4, 5) and logits.shape == (1, 4, 5, 200)
    assert torch.isfinite(xd.grad).all()


def test_densenet_config_depth_fp16(device):
    """BASELINE configs[4] (DenseNet-161, 30 prototypes/class, fp16): the depth is not stated
    (the add-on maps the 1024-channel features to prototype_shape[1]); at the full 1024 the layer
    runs on the wide family, which reads the fp16 feature maps in its GEMM stages (no widening
    pass) and writes g_x in fp16."""
    from protoseg_amd import ops
    B, C, h, w, P, K = 2, 1024, 8, 8, 570, 19
    x, protos, w_last, g_logits, _ = _inputs(B, C, h, w, P, K, seed=161)
    xh = x.half()
    xd = xh.to(device).requires_grad_(True)
    pd = protos.to(device).requires_grad_(True)
    wd = w_last.to(device).requires_grad_(True)
    dist, logits, _ = ops.prototype_layer(xd, pd, wd)
    logits.backward(g_logits.to(device))
    r_logits, r_dist, r_gx, r_gp, r_gw = po.forward_backward(xh.float(), protos, w_last, g_logits, None)
    floor = 1e-6 * ((xh.float() ** 2).sum(1).max() + (protos ** 2).sum(1).max()).item()
    derr = (dist.detach().cpu() - r_dist).abs()
    assert bool((derr <= 1e-4 * r_dist.abs() + floor).all()), f"distances: max err {derr.max().item():.3e}"
    _close(logits, r_logits, "logits")
    assert xd.grad.dtype == torch.float16
    _close(xd.grad.float(), r_gx, "g_x (fp16)", rel=2e-3)
    _close(pd.grad, r_gp, "g_protos")
    _close(wd.grad, r_gw, "g_w")


@pytest.mark.parametrize("precision", ["f32", "bf16x6"])
def test_fp16_native_matches_widened(device, precision):
    """With exact-f32-class products (F32 / BF16X6 requests) the wide family's native fp16 read
    (PROTOSEG_F16) gives the same bits as the f32 path on the exactly widened map: distances,
    logits, g_protos, g_w, and g_x rounded to fp16 once. (BF16X3 requests on fp16 maps take the
    fp16 MFMA distance GEMM: test_fp16_distance_gemm_*.)"""
    from protoseg_amd import ops
    B, C, h, w, P, K = 2, 256, 6, 7, 95, 19
    x, protos, w_last, g_logits, _ = _inputs(B, C, h, w, P, K, seed=5)
    assert ops.x_dtype_supported(C, P, K, torch.float16)
    assert not ops.x_dtype_supported(64, 190, 19, torch.float16)  # C = 64 family: widened
    xh = x.half().to(device)
    outs = []
    for xin in (xh, xh.float()):
        xd = xin.clone().requires_grad_(True)
        pd = protos.to(device).requires_grad_(True)
        wd = w_last.to(device).requires_grad_(True)
        dist, logits, _ = ops.prototype_layer(xd, pd, wd, precision=precision)
        logits.backward(g_logits.to(device))
        outs.append((dist.detach(), logits.detach(), xd.grad.half(), pd.grad, wd.grad))
    torch.cuda.synchronize()
    for name, a, b in zip(("dist", "logits", "g_x", "g_protos", "g_w"), outs[0], outs[1]):
        assert torch.equal(a, b), name


def _f32_bound(x, protos):
    """f32 rounding bound of the expanded distance x2 + p2 - 2 x.p over C f32 sums:
    2e-6 (||x||^2 + ||p||^2). bf16x3 products (3 x 2^-16 per product) exceed it about 8x at C = 1024."""
    return 2e-6 * ((x.double() ** 2).sum(1)[:, None] + (protos.double() ** 2).sum(1)[None, :, None, None])


@pytest.mark.parametrize("B,C,h,w,P,K", [
    (2, 1024, 16, 16, 570, 19),  # BASELINE configs[4]: DenseNet depth, 30 prototypes/class
    (1, 200, 9, 8, 77, 7),       # ragged: C % 32, P % 192, pixels % 128 all non-zero
    (3, 96, 4, 6, 400, 40),      # pixel tiles straddling images (HW = 24)
])
def test_fp16_distance_gemm_vs_float64(device, B, C, h, w, P, K):
    """The fp16 distance GEMM (wide_dist_f16_kernel: x exact in fp16, prototypes scaled by a power
    of two and split into two fp16 terms, v_mfma_f32_32x32x16_f16) against float64 distances: within
    the f32 rounding bound of the expanded form, i.e. as accurate as exact f32 products (bf16x3
    products would not meet this bound at C = 1024). Prototypes with large and tiny entries exercise
    the per-row scale. Logits against the oracle on the fp16 map."""
    from protoseg_amd import ops
    x, protos, w_last, g_logits, _ = _inputs(B, C, h, w, P, K, seed=C + P)
    protos[::5] *= 3000.0      # rows far above fp16's comfortable range before scaling
    protos[1::5] *= 1e-3       # and far below it
    xh = x.half()
    dist, logits, _ = ops.prototype_layer(xh.to(device), protos.to(device), w_last.to(device))
    torch.cuda.synchronize()
    xd = xh.double()
    ref = ((xd[:, None] - protos.double()[None, :, :, None, None]) ** 2).sum(2)
    err = (dist.double().cpu() - ref).abs()
    assert bool((err <= _f32_bound(xh.float(), protos)).all()), f"max err {err.max().item():.3e}"
    r_logits = po.forward_from_conv_features(xh.float(), protos[:, :, None, None], w_last)[0]
    _close(logits, r_logits, "logits", rel=1e-4)


def test_fp16_distance_gemm_near_zero(device):
    """configs[4] depth with every prototype copied from a feature-map patch (d ~ 0, the state right
    after push): the fp16 GEMM's distances stay within the f32 rounding bound of float64, as the
    exact-f32 path's do, and its log activations are log((d+1)/(d+1e-4)) of those distances."""
    from protoseg_amd import ops
    B, C, h, w, P, K = 2, 1024, 16, 16, 570, 19
    x, _, w_last, _, _ = _inputs(B, C, h, w, P, K, seed=7)
    xh = x.half()
    flat = xh.float().permute(0, 2, 3, 1).reshape(-1, C)
    protos = flat[torch.randint(0, flat.shape[0], (P,), generator=torch.Generator().manual_seed(1))].clone()
    xd, pd, wd = xh.to(device), protos.to(device), w_last.to(device)
    ref = ((xh.double()[:, None] - protos.double()[None, :, :, None, None]) ** 2).sum(2)
    bound = _f32_bound(xh.float(), protos)
    assert int((ref == 0).sum()) >= P  # every prototype has an exact match
    for prec in ("bf16x3", "f32"):  # bf16x3 requests take the fp16 GEMM; f32 the exact f32 path
        dist, _, act = ops.prototype_layer(xd, pd, wd, with_act=True, precision=prec)
        torch.cuda.synchronize()
        err = (dist.double().cpu() - ref).abs()
        assert bool((err <= bound).all()), f"{prec}: max err {err.max().item():.3e}"
        d = dist.double().cpu().permute(0, 2, 3, 1).reshape(-1, P)
        r_act = torch.log((d + 1) / (d + 1e-4))
        _close(act.double().cpu().reshape(-1, P), r_act, f"{prec} act", rel=1e-5)


def test_wide_backward_from_saved_distances(device):
    """protoseg_l2_bwd_saved (the wide family reads the forward's distances instead of
    recomputing them) gives the recomputing backward's gradients bit for bit, and the autograd
    op saves the distances for it."""
    from protoseg_amd import ops
    B, C, h, w, P, K = 2, 256, 6, 7, 95, 19
    x, protos, w_last, g_logits, _ = _inputs(B, C, h, w, P, K, seed=21)
    prec = ops.precision_code(None)
    assert ops.bwd_reads_dist(C, P, K, prec) and not ops.bwd_reads_dist(64, 361, 19, prec)
    xd, pd, wd, gl = x.to(device), protos.to(device), w_last.to(device), g_logits.to(device)
    dist = ops.l2_forward(xd, pd, wd, 1e-4, 0, prec, True, True, False)[0]
    a = ops.l2_backward(xd, pd, wd, gl, None, 1e-4, 0, prec, True, True, True)
    b = ops.l2_backward(xd, pd, wd, gl, None, 1e-4, 0, prec, True, True, True, None, dist)
    torch.cuda.synchronize()
    for name, u, v in zip(("g_x", "g_p", "g_w"), a, b):
        assert torch.equal(u, v), name
    xr = xd.clone().requires_grad_(True)
    pr = pd.clone().requires_grad_(True)
    wr = wd.clone().requires_grad_(True)
    dist2, logits, _ = ops.prototype_layer(xr, pr, wr)
    logits.backward(gl)
    torch.cuda.synchronize()
    assert torch.equal(dist2, dist)
    assert torch.equal(xr.grad, a[0]) and torch.equal(pr.grad, a[1]) and torch.equal(wr.grad, a[2])
