"""ORACLE — test infrastructure only. CPU restatement of the reference's KLD similarity loss.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline; the product path never calls it.

Restates segmentation/module.py:167-208 op for op (torch CPU, float32), quirks included:
  * ``patch_activations`` is the SECOND output of PPNet.forward, i.e. the distances
    [B, P, h, w] (model.py:283), permuted / reshaped to [B, h*w, P] (module.py:153-154);
  * ``target_img`` is the resized label BEFORE the void shift (module.py:150): raw label
    values with 0 = void. The prototype column used for label value c is c itself
    (module.py:170-178), so void pixels pair with class-0 prototypes and the label value
    ``num_classes`` is skipped (module.py:171). Kept as-is for parity;
  * per (image, class): log_softmax over the masked pixels of each prototype of the class,
    then the symmetric KL of every prototype pair i < j (module.py:180-200); a class with
    fewer than 2 prototypes or fewer than 2 pixels contributes nothing (module.py:186);
  * loss = mean over all pairs of exp(-kld) (module.py:202-206), 0.0 without pairs.
The gradient is torch autograd of the same ops.

Parity status: UNPINNED against the reference itself (import denied; the
reference ships no tests). Pinned by tests/test_kld_oracle.py against an
independent float64 closed form and frozen as tests/golden/kld_small.npz.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
import torch.nn.functional as F


def kld_loss(distances: torch.Tensor, target_img: torch.Tensor, prototype_class_identity: torch.Tensor):
    """module.py:167-208. distances [B, P, h, w] f32; target_img [B, h*w] int; identity [P, K].
    Returns (kld_loss: tensor or 0.0, number of pairs)."""
    patch_activations = distances.permute(0, 2, 3, 1)                                      # module.py:153
    patch_activations_img = patch_activations.reshape(patch_activations.shape[0], -1,
                                                      patch_activations.shape[-1])         # module.py:154
    kld_terms = []
    for img_i in range(len(target_img)):                                                   # module.py:169
        for cls_i in torch.unique(target_img[img_i]).cpu().detach().numpy():              # module.py:170
            if cls_i < 0 or cls_i >= prototype_class_identity.shape[1]:                    # module.py:171
                continue
            cls_protos = torch.nonzero(prototype_class_identity[:, cls_i]).flatten().cpu().detach().numpy()
            if len(cls_protos) == 0:                                                       # module.py:175
                continue
            cls_mask = (target_img[img_i] == cls_i)                                        # module.py:178
            log_cls_activations = [torch.masked_select(patch_activations_img[img_i, :, i], cls_mask)
                                   for i in cls_protos]                                    # module.py:180-181
            log_cls_activations = [F.log_softmax(act, dim=0) for act in log_cls_activations]
            for i in range(len(cls_protos)):                                               # module.py:185
                if len(cls_protos) < 2 or len(log_cls_activations[0]) < 2:
                    continue
                log_p1_scores = log_cls_activations[i]
                for j in range(i + 1, len(cls_protos)):
                    log_p2_scores = log_cls_activations[j]
                    kld1 = F.kl_div(log_p1_scores, log_p2_scores, log_target=True, reduction="sum")
                    kld2 = F.kl_div(log_p2_scores, log_p1_scores, log_target=True, reduction="sum")
                    kld_terms.append((kld1 + kld2) / 2.0)                                  # module.py:199-200
    if len(kld_terms) > 0:                                                                 # module.py:202-206
        return torch.mean(torch.exp(-torch.stack(kld_terms))), len(kld_terms)
    return 0.0, 0


def kld_loss_and_grad(distances: torch.Tensor, target_img: torch.Tensor, prototype_class_identity: torch.Tensor,
                      g_loss: float = 1.0) -> Tuple[float, int, torch.Tensor]:
    """(loss, n_pairs, d(g_loss * loss) / d distances) by autograd of kld_loss."""
    d = distances.detach().float().clone().requires_grad_(True)
    loss, n = kld_loss(d, target_img, prototype_class_identity)
    if n == 0:
        return 0.0, 0, torch.zeros_like(d)
    (loss * g_loss).backward()
    return float(loss.detach()), n, d.grad.detach()


def kld_loss_float64(distances: np.ndarray, target_img: np.ndarray, proto_class: np.ndarray, K: int):
    """Independent float64 closed form (numpy) of the same loss and its gradient, used to pin
    the restatement: symKL_ij = (KL(p_i||p_j) + KL(p_j||p_i)) / 2, L = mean exp(-symKL),
    dL/dz_i = sum_j w_ij (p_i (lp_i - lp_j - KL(p_i||p_j) + 1) - p_j) / 2 with
    w_ij = -exp(-symKL_ij) / N."""
    B, P = distances.shape[:2]
    d = distances.reshape(B, P, -1).astype(np.float64)
    terms, groups = [], []
    for b in range(B):
        for c in np.unique(target_img[b]):
            if c < 0 or c >= K:
                continue
            protos = np.nonzero(proto_class == c)[0]
            mask = target_img[b] == c
            if len(protos) < 2 or mask.sum() < 2:
                continue
            z = d[b][protos][:, mask]
            lp = z - z.max(1, keepdims=True)
            lp = lp - np.log(np.exp(lp).sum(1, keepdims=True))
            p = np.exp(lp)
            kl = (p[:, None, :] * (lp[:, None, :] - lp[None, :, :])).sum(-1)   # kl[i, j] = KL(p_i || p_j)
            groups.append((b, protos, mask, p, lp, kl))
            for i in range(len(protos)):
                for j in range(i + 1, len(protos)):
                    terms.append(0.5 * (kl[i, j] + kl[j, i]))
    grad = np.zeros_like(d)
    if not terms:
        return 0.0, 0, grad.reshape(distances.shape)
    n = len(terms)
    loss = float(np.mean(np.exp(-np.asarray(terms))))
    for b, protos, mask, p, lp, kl in groups:
        w = -np.exp(-0.5 * (kl + kl.T)) / n
        np.fill_diagonal(w, 0.0)
        g = np.zeros_like(p)
        for i in range(len(protos)):
            for j in range(len(protos)):
                if i != j:
                    g[i] += w[i, j] * 0.5 * (p[i] * (lp[i] - lp[j] - kl[i, j] + 1.0) - p[j])
        for i, proto in enumerate(protos):
            grad[b, proto, mask] = g[i]
    return loss, n, grad.reshape(distances.shape)


def synthetic_targets(B: int, h: int, w: int, K: int, seed: int = 20220227, block: int = 4) -> torch.Tensor:
    """Label maps [B, h*w] int64 in 0..K (0 = void) made of square blocks, like a resized
    Cityscapes label (module.py:143-146): contiguous regions, every value possible."""
    gen = torch.Generator().manual_seed(seed)
    bh, bw = (h + block - 1) // block, (w + block - 1) // block
    coarse = torch.randint(0, K + 1, (B, bh, bw), generator=gen)
    full = coarse.repeat_interleave(block, 1).repeat_interleave(block, 2)[:, :h, :w]
    return full.reshape(B, h * w).contiguous()
