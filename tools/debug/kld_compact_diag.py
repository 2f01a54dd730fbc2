"""Diagnose test_compact_expands_to_dense failing after large-shape tests: fill the caching
allocator with garbage first, then compare compact-expanded vs dense and report mismatches."""
import sys
import os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."),
                os.path.join(os.path.dirname(__file__), "..", "..", "adlm-inherently-interpretable-segmentation_amd")]
import torch
from oracle import kld_oracle as ko
from oracle import protoseg_oracle as po
from protoseg_amd import kld, ops

dev = torch.device("cuda:0")
for fill in (False, True):
    if fill:  # garbage in freed blocks of many sizes
        bufs = [torch.full((n,), float("nan"), device=dev) for n in (1 << 10, 1 << 14, 1 << 18, 1 << 22, 1 << 24)]
        bufs += [torch.randint(-2**31, 2**31 - 1, (n,), device=dev, dtype=torch.int32) for n in (1 << 12, 1 << 16, 1 << 20)]
        del bufs
    B, h, w, P, K, block = 2, 9, 11, 38, 19, 3
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed=B * 5 + P)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1)).to(dev)
    target = ko.synthetic_targets(B, h, w, K, seed=h + w, block=block).to(dev)
    ident = po.class_identity(P, K)
    cols, mpc = kld.prototype_columns(ident, dev)
    loss, npairs, ws = torch.ops.protoseg.kld_forward(dist, target, cols, K, mpc)
    g_loss = torch.full((), 0.25, device=dev)
    dense = torch.ops.protoseg.kld_backward(dist, target, cols, K, mpc, ws, g_loss)
    g_cls, pix_cls, proto_slot = kld.kld_backward_compact(dist, target, cols, K, mpc, ws, g_loss)
    exp = ops.expand_compact((g_cls, pix_cls, proto_slot, mpc), B, P, h * w).reshape(B, P, h, w)
    torch.cuda.synchronize()
    bad = (exp != dense) & ~(torch.isnan(exp) & torch.isnan(dense))
    nn = int(torch.isnan(dense).sum()), int(torch.isnan(exp).sum())
    print(f"fill={fill} equal={torch.equal(exp, dense)} mismatches={int(bad.sum())} nan(dense,exp)={nn} mpc={mpc} loss={float(loss):.6f} npairs={int(npairs)}")
    idx = bad.nonzero()[:10].tolist()
    t = target.reshape(B, -1).cpu()
    pc = pix_cls.reshape(B, -1).cpu()
    sl = proto_slot.cpu()
    for b, p, i, j in idx:
        n = i * w + j
        print(f"  b={b} p={p} n={n} label={int(t[b, n])} col={int(cols[p])} slot={int(sl[p])} pix_cls={int(pc[b, n])} "
              f"dense={float(dense[b, p, i, j]):.6g} exp={float(exp[b, p, i, j]):.6g}")
