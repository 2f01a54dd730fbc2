"""ORACLE — test infrastructure only. CPU restatement of the reference's prototype layer.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline; the product path never calls it.

Parity status: the reference's Python cannot be imported or run here (denied)
and it ships no tests, fixtures or golden vectors for this path. This is
therefore an op-for-op restatement of the reference's own code, pinned by analytic
known-answer checks (tests/test_oracle.py) and frozen as committed golden vectors
(tests/golden/). Parity against the reference binary itself is UNPINNED.

Op order follows the reference exactly (torch CPU, float32):
  model.py:203-221  _l2_convolution:  x**2 -> conv2d(x2, ones) ; sum(p**2) ; conv2d(x, P)
                                       -> -2*xp + p2 -> + x2_patch_sum -> relu
  model.py:231-237  distance_2_similarity: log((d + 1) / (d + eps)) | -d
  model.py:259-283  forward_from_conv_features (patch classification): permute(0,2,3,1)
                    -> reshape(-1, P) -> activation -> last_layer (Linear, no bias)
                    -> reshape(B, h, w, K); returns (logits, distances)
  backward: torch autograd of the above (the reference has no custom backward)
  model.py:54, 66-71, 359-371, 386: initialisation (U[0,1) prototypes, class identity,
                    last layer 1 / incorrect_strength).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

EPSILON = 1e-4  # model.py:50


def l2_convolution(x: torch.Tensor, prototype_vectors: torch.Tensor, ones: torch.Tensor) -> torch.Tensor:
    """model.py:203-221"""
    x2 = x ** 2
    x2_patch_sum = F.conv2d(input=x2, weight=ones)
    p2 = prototype_vectors ** 2
    p2 = torch.sum(p2, dim=(1, 2, 3))
    p2_reshape = p2.view(-1, 1, 1)
    xp = F.conv2d(input=x, weight=prototype_vectors)
    intermediate_result = -2 * xp + p2_reshape
    return F.relu(x2_patch_sum + intermediate_result)


def distance_2_similarity(distances: torch.Tensor, activation: str = "log", epsilon: float = EPSILON):
    """model.py:231-237"""
    if activation == "log":
        return torch.log((distances + 1) / (distances + epsilon))
    if activation == "linear":
        return -distances
    raise ValueError(activation)


def forward_from_conv_features(x, prototype_vectors, last_layer_weight, activation="log", epsilon=EPSILON,
                               return_activations=False):
    """model.py:259-283 (patch_classification=True)."""
    if prototype_vectors.dim() == 2:
        prototype_vectors = prototype_vectors[:, :, None, None]
    ones = torch.ones_like(prototype_vectors)
    distances = l2_convolution(x, prototype_vectors, ones)
    batch_size, num_prototypes, rows, cols = distances.shape
    dist_view = distances.permute(0, 2, 3, 1).contiguous().reshape(-1, num_prototypes)
    activations = distance_2_similarity(dist_view, activation, epsilon)
    logits = F.linear(activations, last_layer_weight)  # nn.Linear(bias=False), model.py:143-144
    logits = logits.reshape(batch_size, rows, cols, -1)
    if return_activations:
        return logits, activations
    return logits, distances


def forward_backward(x, prototype_vectors, last_layer_weight, g_logits: Optional[torch.Tensor],
                     g_dist: Optional[torch.Tensor], activation="log", epsilon=EPSILON
                     ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """Autograd of forward_from_conv_features. Returns (logits, distances, g_x, g_protos [P,C], g_w)."""
    x = x.detach().float().clone().requires_grad_(True)
    protos = prototype_vectors.detach().float().reshape(prototype_vectors.shape[0], -1, 1, 1).clone()
    protos.requires_grad_(True)
    w = last_layer_weight.detach().float().clone().requires_grad_(True)
    logits, distances = forward_from_conv_features(x, protos, w, activation, epsilon)
    outs, grads = [], []
    if g_logits is not None:
        outs.append(logits)
        grads.append(g_logits.float())
    if g_dist is not None:
        outs.append(distances)
        grads.append(g_dist.float())
    torch.autograd.backward(outs, grads)
    g_w = w.grad if g_logits is not None else None
    return (logits.detach(), distances.detach(), x.grad.detach(), protos.grad.detach().reshape(protos.shape[0], -1),
            None if g_w is None else g_w.detach())


def class_identity(num_prototypes: int, num_classes: int) -> torch.Tensor:
    """model.py:66-71"""
    identity = torch.zeros(num_prototypes, num_classes)
    per_class = num_prototypes // num_classes
    for i in range(num_classes):
        identity[i * per_class:(i + 1) * per_class, i] = 1
    return identity


def last_layer_init(identity: torch.Tensor, incorrect_strength: float = -0.5) -> torch.Tensor:
    """model.py:359-371"""
    positive = torch.t(identity)
    return 1 * positive + incorrect_strength * (1 - positive)


def synthetic_inputs(B: int, C: int, h: int, w: int, P: int, K: int, seed: int = 20220227,
                     dtype=torch.float32):
    """SURVEY.md §8d synthetic tensors: X = sigmoid(N(0, 2^2)) (the deeplab_simple add-on
    output lies in [0, 1]), prototypes U[0,1) (model.py:54), last layer from the class identity."""
    gen = torch.Generator().manual_seed(seed)
    x = torch.sigmoid(2.0 * torch.randn(B, C, h, w, generator=gen)).to(dtype)
    protos = torch.rand(P, C, generator=gen)
    w_last = last_layer_init(class_identity(P, K))
    return x, protos, w_last
