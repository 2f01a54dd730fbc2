"""The training backward that serves up to 384 prototypes per launch, against the oracle's autograd
of model.py:203-283 and against the 192-prototype fused kernel:
  wave     l2_bwd_wave.hip: 4 waves, one per SIMD, each owning a quarter of the prototypes for
           every product, 32x32x16 bf16 MFMA (bf16x3 products).
protoseg_set_backward_kernel (the bwd_kernel fixture) selects the kernel per call (wave / fused).
Tolerance: rtol 1e-4 of each gradient's own scale, as tests/test_gpu_l2.py."""

KERNELS = ["wave"]
import pytest
import torch

from oracle import protoseg_oracle as po

pytestmark = pytest.mark.gpu


def _ops():
    from protoseg_amd import ops
    return ops


def assert_scaled_close(a, ref, rtol=1e-4, name=""):
    a, ref = a.double().cpu(), ref.double().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (a - ref).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} > {rtol:g} * scale {scale:.3e}"


@pytest.mark.parametrize("B,h,w,P,K", [
    (2, 17, 17, 38, 19),     # one 32-prototype block (Pp 128)
    (1, 9, 11, 100, 5),      # ragged pixel tail, 5 classes
    (2, 65, 65, 190, 19),    # cityscapes_*_imnet.gin, 10 prototypes/class (Pp 256)
    (2, 41, 41, 210, 21),    # pascal: 21 classes
    (1, 65, 65, 361, 19),    # the metric's 19 prototypes/class (Pp 384, one pass)
    (1, 33, 35, 384, 32),    # full Pp, K = 32
    (1, 16, 16, 570, 19),    # two chunks of 285 (g_x accumulated by the second)
])
@pytest.mark.parametrize("activation", ["log", "linear"])
@pytest.mark.parametrize("kernel", KERNELS)
def test_wave_backward_vs_oracle(device, bwd_kernel, B, h, w, P, K, activation, kernel):
    bwd_kernel(kernel)
    ops = _ops()
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=B * 100 + h + P)
    gen = torch.Generator().manual_seed(11)
    w_last = w_last + 0.05 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    _, _, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, None, activation)
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device), g_logits.to(device), None,
                                 1e-4, ops.ACT_KINDS[activation], ops.PRECISIONS["bf16x3"], True, True, True)
    torch.cuda.synchronize()
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("P", [190, 361])
@pytest.mark.parametrize("kernel", KERNELS)
def test_wave_backward_with_g_dist(device, bwd_kernel, P, kernel):
    bwd_kernel(kernel)
    ops = _ops()
    B, h, w, K = 2, 33, 31, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=P)
    gen = torch.Generator().manual_seed(3)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = 0.01 * torch.randn(B, P, h, w, generator=gen)
    _, _, ref_gx, ref_gp, ref_gw = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    gx, gp, gw = ops.l2_backward(x.to(device), protos.to(device), w_last.to(device), g_logits.to(device),
                                 g_dist.to(device), 1e-4, 0, ops.PRECISIONS["bf16x3"], True, True, True)
    torch.cuda.synchronize()
    assert_scaled_close(gx, ref_gx, 1e-4, "g_x")
    assert_scaled_close(gp, ref_gp, 1e-4, "g_protos")
    assert_scaled_close(gw, ref_gw, 1e-4, "g_w")


@pytest.mark.parametrize("P", [190, 361])
@pytest.mark.parametrize("kernel", KERNELS)
def test_wave_equals_fused_within_rounding(device, bwd_kernel, P, kernel):
    """The same gradients from both kernels (different MFMA shapes and summation orders)."""
    ops = _ops()
    B, h, w, K = 4, 65, 65, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=7 + P)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(2))
    args = (x.to(device), protos.to(device), w_last.to(device), g_logits.to(device), None, 1e-4, 0,
            ops.PRECISIONS["bf16x3"], True, True, True)
    bwd_kernel("fused")
    a = ops.l2_backward(*args)
    bwd_kernel(kernel)
    b = ops.l2_backward(*args)
    torch.cuda.synchronize()
    for u, v, name in zip(a, b, ("g_x", "g_protos", "g_w")):
        assert_scaled_close(v, u, 2e-5, name)


@pytest.mark.parametrize("kernel", KERNELS)
def test_wave_deterministic(device, bwd_kernel, kernel):
    bwd_kernel(kernel)
    ops = _ops()
    B, h, w, P, K = 8, 65, 65, 361, 19
    x, protos, w_last = po.synthetic_inputs(B, 64, h, w, P, K, seed=1)
    g_logits = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(4))
    args = (x.to(device), protos.to(device), w_last.to(device), g_logits.to(device), None, 1e-4, 0,
            ops.PRECISIONS["bf16x3"], True, True, True)
    a = ops.l2_backward(*args)
    b = ops.l2_backward(*args)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kernel", KERNELS)
def test_wave_x_sigmoid_and_bf16_features(device, bwd_kernel, xdtype, kernel):
    from protoseg_amd import _lib
    """PROTOSEG_X_SIGMOID (the add-on nn.Sigmoid on the x load) and bf16 feature maps at P = 361:
    against the oracle on sigmoid(pre-activation), gradient taken w.r.t. the pre-activation."""
    bwd_kernel("wave")
    ops = _ops()
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
    gx, gp, gw = ops.l2_backward(pre.to(device), protos.to(device), w_last.to(device), g_logits.to(device), None,
                                 1e-4, ops.ACT_KINDS["log"] | _lib.X_SIGMOID, ops.PRECISIONS["bf16x3"], True, True,
                                 True)
    torch.cuda.synchronize()
    tol = 1e-4 if xdtype == torch.float32 else 1e-2  # bf16 g_x output rounding
    assert_scaled_close(gx.float(), pre_ref.grad, tol, "g_pre")
    assert_scaled_close(gp, protos_ref.grad, 1e-4, "g_protos")
    assert_scaled_close(gw, w_ref.grad, 1e-4, "g_w")
