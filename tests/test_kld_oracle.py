"""CPU: pin the KLD oracle (module.py:167-208 restated) before trusting it — an independent
float64 closed form, the committed golden vector, the reference's skip rules; and the host side
of the HIP wrapper (class columns, argument validation without a GPU)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import kld_oracle as ko
from oracle import protoseg_oracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _case(B, h, w, P, K, seed, block=3):
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1))
    return dist, ko.synthetic_targets(B, h, w, K, seed + 1, block), po.class_identity(P, K)


@pytest.mark.parametrize("B,h,w,P,K", [(2, 9, 11, 38, 19), (1, 13, 7, 30, 3), (3, 6, 6, 10, 5)])
def test_oracle_matches_float64_closed_form(B, h, w, P, K):
    dist, target, ident = _case(B, h, w, P, K, seed=B + h + P)
    loss, n, g = ko.kld_loss_and_grad(dist, target, ident)
    l64, n64, g64 = ko.kld_loss_float64(dist.numpy(), target.numpy(), ident.argmax(1).numpy(), K)
    assert n == n64 and n > 0
    assert abs(loss - l64) <= 1e-6 * max(1.0, abs(l64))
    assert np.abs(g.numpy() - g64).max() <= 1e-5 * np.abs(g64).max()


def test_oracle_reproduces_golden():
    g = np.load(os.path.join(GOLDEN, "kld_small.npz"))
    K = int(g["num_classes"])
    ident = torch.nn.functional.one_hot(torch.from_numpy(g["proto_class"]).long(), K).float()
    loss, n, grad = ko.kld_loss_and_grad(torch.from_numpy(g["dist"]), torch.from_numpy(g["target"]), ident)
    assert n == int(g["n_pairs"])
    assert abs(loss - float(g["loss"])) <= 1e-6
    assert np.allclose(grad.numpy(), g["g_dist"], rtol=1e-5, atol=1e-6 * np.abs(g["g_dist"]).max())


def test_reference_skip_rules():
    """module.py:171 (value K skipped), 186 (< 2 pixels / < 2 prototypes), 207 (no pair -> 0)."""
    P, K, h, w = 6, 3, 4, 4
    dist = torch.rand(1, P, h, w)
    ident = po.class_identity(P, K)
    only_k = torch.full((1, h * w), K)                     # every pixel has the skipped value K
    assert ko.kld_loss(dist, only_k, ident) == (0.0, 0)
    single = torch.full((1, h * w), K)
    single[0, 3] = 1                                       # class 1 has one pixel
    assert ko.kld_loss(dist, single, ident) == (0.0, 0)
    void = torch.zeros(1, h * w, dtype=torch.long)         # void pixels pair with class-0 prototypes
    loss, n = ko.kld_loss(dist, void, ident)
    assert n == 1 and 0.0 < float(loss) <= 1.0
    one_proto = po.class_identity(3, 3)                    # one prototype per class: no pair
    assert ko.kld_loss(torch.rand(1, 3, h, w), void, one_proto) == (0.0, 0)


def test_identical_distributions_give_loss_one():
    """Known answer: prototypes with equal distance maps -> KL = 0 -> exp(0) = 1, zero gradient."""
    h = w = 5
    base = torch.rand(1, 1, h, w)
    dist = base.repeat(1, 4, 1, 1)
    ident = po.class_identity(4, 2)
    target = torch.ones(1, h * w, dtype=torch.long)
    target[0, :7] = 0
    loss, n, g = ko.kld_loss_and_grad(dist, target, ident)
    assert n == 2 and abs(loss - 1.0) < 1e-6
    assert g.abs().max().item() < 1e-6


def test_prototype_columns_host_logic():
    from protoseg_amd import ProtosegError
    from protoseg_amd.kld import prototype_columns
    ident = po.class_identity(190, 19)
    cols, mpc = prototype_columns(ident, "cpu")
    assert mpc == 10 and torch.equal(cols, (torch.arange(190) // 10).to(torch.int32))
    two_hot = ident.clone()
    two_hot[0, 5] = 1
    with pytest.raises(ProtosegError):
        prototype_columns(two_hot, "cpu")
    with pytest.raises(ProtosegError):
        prototype_columns(po.class_identity(66, 2), "cpu")   # 33 prototypes in one class


def test_kld_abi_validation_without_gpu():
    from protoseg_amd import _lib
    lib = _lib.load()
    null, dummy = ctypes.c_void_p(None), ctypes.c_void_p(256)
    n = lib.protoseg_kld_workspace_size(32, 190, 4225, 19)
    assert n > 0 and n % 256 == 0
    assert lib.protoseg_kld_workspace_size(0, 190, 4225, 19) == 0
    st = lib.protoseg_kld_forward(null, 2, 38, 10, dummy, _lib.I64, dummy, 19, 2, dummy, null, dummy, n, null)
    assert st == _lib.ERR_INVALID
    st = lib.protoseg_kld_forward(dummy, 2, 38, 10, dummy, _lib.I64, dummy, 19, 33, dummy, null, dummy, n, null)
    assert st == _lib.ERR_UNSUPPORTED and b"max_per_class" in lib.protoseg_last_error()
    st = lib.protoseg_kld_forward(dummy, 2, 38, 10, dummy, _lib.I64, dummy, 64, 2, dummy, null, dummy, 1 << 30, null)
    assert st == _lib.ERR_UNSUPPORTED
    st = lib.protoseg_kld_forward(dummy, 2, 38, 10, dummy, _lib.F32, dummy, 19, 2, dummy, null, dummy, n, null)
    assert st == _lib.ERR_UNSUPPORTED
    st = lib.protoseg_kld_backward(dummy, 2, 38, 10, dummy, _lib.I64, dummy, 19, 2, null, dummy, 16, dummy, null)
    assert st == _lib.ERR_INVALID and b"workspace" in lib.protoseg_last_error()


def test_eval_oracle_metrics_and_abi():
    """eval_valid.py:216-219 formulas on hand counts; the eval C ABI validates without a GPU."""
    from oracle import eval_oracle as eo
    from protoseg_amd import _lib
    acc, miou, ious = eo.metrics(30, 40, np.array([10, 0, 5]), np.array([20, 0, 10]))
    assert acc == 75.0 and ious == {0: 50.0, 2: 50.0} and miou == 50.0
    lib = _lib.load()
    null, dummy = ctypes.c_void_p(None), ctypes.c_void_p(256)
    st = lib.protoseg_eval_counts(null, null, 1, 4, 4, 19, 0, dummy, _lib.I64, 8, 8, null, 0, null, dummy, null)
    assert st == _lib.ERR_INVALID
    st = lib.protoseg_eval_counts(dummy, dummy, 1, 4, 4, 19, 10, dummy, _lib.I64, 8, 8, null, 0, null, dummy, null)
    assert st == _lib.ERR_INVALID and b"proto_class" in lib.protoseg_last_error()
    st = lib.protoseg_eval_counts(dummy, null, 1, 4, 4, 65, 0, dummy, _lib.I64, 8, 8, null, 0, null, dummy, null)
    assert st == _lib.ERR_UNSUPPORTED
