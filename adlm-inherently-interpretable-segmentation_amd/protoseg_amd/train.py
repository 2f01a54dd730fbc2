"""Data-parallel training step of the patch-classification model.

Mirrors reference segmentation/module.py:118-260 (``PatchClassificationModule._step``, train
branch): the label map is resized to the logits' grid (dataset.py:23-31), cross entropy over
the non-void pixels (module.py:152-163), the KLD prototype-diversity term (module.py:165-208,
``kld.kld_loss``), the L1 penalty on the last layer's off-class weights (module.py:214-219),
``loss / iter_size`` backward, and ``optimizer.step()`` every ``iter_size`` micro-steps
(module.py:235-243). Multi-scale outputs (a list) are averaged as in module.py:226.

Data parallelism (one process per GPU, RCCL): every rank runs its own micro-batch. So that the
result equals ONE process stepping on the concatenated batch (not just a mean of per-rank
means — the non-void pixel counts and the KLD pair counts differ between ranks), each micro-step
all-reduces its two counts (a 2-element collective), scales its loss sums by the global counts
and the L1 term by 1 / world, and the gradients are SUMMED over ranks by ``GradientBuckets`` on
the accumulation boundary only, with the bucket all-reduces launched from backward's gradient
hooks (overlapping the rest of the backward). Micro-steps inside an accumulation exchange
nothing but the counts.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import Tensor

from .distributed import GradientBuckets, world_info


def backbone_params(features, key: str):
    """segmentation/utils.py:42-61 (``get_params``): "1x" = the conv parameters of the ResNet
    layers, "10x" / "20x" = the ASPP conv weights / biases."""
    for name, m in features.named_modules():
        if not isinstance(m, torch.nn.Conv2d):
            continue
        if key == "1x" and "layer" in name:
            yield from m.parameters()
        elif key == "10x" and "aspp" in name:
            yield m.weight
        elif key == "20x" and "aspp" in name:
            yield m.bias


def joint_param_groups(ppnet, lr_features: float = 2.5e-5, lr_add_on_layers: float = 2.5e-4,
                       lr_prototype_vectors: float = 2.5e-4, weight_decay: float = 5e-4):
    """The joint-phase optimizer groups of module.py:357-382 (defaults: cityscapes_*_imnet.gin
    joint_optimizer_*): backbone 1x / 10x / 20x, add-on layers, prototype vectors (no weight
    decay). BatchNorm and the last layer get gradients but are not stepped, as in the reference."""
    wd = weight_decay
    return [
        {"params": list(backbone_params(ppnet.features, "1x")), "lr": lr_features, "weight_decay": wd},
        {"params": list(backbone_params(ppnet.features, "10x")), "lr": 10 * lr_features, "weight_decay": wd},
        {"params": list(backbone_params(ppnet.features, "20x")), "lr": 10 * lr_features, "weight_decay": wd},
        {"params": list(ppnet.add_on_layers.parameters()), "lr": lr_add_on_layers, "weight_decay": wd},
        {"params": [ppnet.prototype_vectors], "lr": lr_prototype_vectors},
    ]


def _default_resize(labels: Tensor, h: int, w: int) -> Tensor:
    from .knn import resize_label
    return resize_label(labels, h, w)


def _default_kld(distances: Tensor, target_img: Tensor, class_identity: Tensor):
    """(loss, n_pairs): module.py:167-208 on the HIP kernels."""
    from .kld import kld_with_pairs, prototype_columns
    cols, mpc = prototype_columns(class_identity, distances.device)
    return kld_with_pairs(distances, target_img, cols, int(class_identity.shape[1]), mpc)


class PatchClassificationStep:
    """One training micro-step of module.py:_step ('train'), data-parallel when torch.distributed
    is initialised (or ``process_group`` is given) with more than one rank.

    ``ppnet(image)`` must return ``(logits [B, h, w, K], distances [B, P, h, w])`` or a list of
    such pairs (PPNet.forward with patch_classification). ``target`` is the label map at image
    resolution [B, H, W] (resized here with PIL-nearest semantics) or already at [B, h, w].
    ``kld_fn(distances, target_img, class_identity) -> (mean loss, n_pairs)`` and
    ``resize_fn(labels, h, w)`` default to the HIP kernels.
    """

    def __init__(self, ppnet, optimizer, loss_weight_crs_ent: float = 1.0, loss_weight_kld: float = 0.0,
                 loss_weight_l1: float = 1e-4, iter_size: int = 1, ignore_void_class: bool = True,
                 lr_scheduler=None, process_group=None, bucket_mb: float = 64.0,
                 kld_fn: Optional[Callable] = None, resize_fn: Optional[Callable] = None):
        self.ppnet = ppnet
        self.optimizer = optimizer
        self.loss_weight_crs_ent = loss_weight_crs_ent
        self.loss_weight_kld = loss_weight_kld
        self.loss_weight_l1 = loss_weight_l1
        self.iter_size = int(iter_size)
        self.ignore_void_class = ignore_void_class
        self.lr_scheduler = lr_scheduler
        self.group = process_group
        self.kld_fn = kld_fn or _default_kld
        self.resize_fn = resize_fn or _default_resize
        self.iter_steps = 0
        # gradients are summed: the per-rank losses are already scaled by the global counts
        self.buckets = GradientBuckets([p for p in ppnet.parameters() if p.requires_grad], bucket_mb,
                                       process_group, average=False)

    def _global(self, t: Tensor) -> Tensor:
        if world_info(self.group)[1] > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def loss(self, image: Tensor, target: Tensor) -> Dict[str, Tensor]:
        """Forward + loss of one micro-batch (module.py:128-228), scaled for the global batch."""
        _, world = world_info(self.group)
        outputs = self.ppnet(image)
        if not isinstance(outputs, list):
            outputs = [outputs]
        identity = self.ppnet.prototype_class_identity.to(image.device)
        if hasattr(self.ppnet, "nearest_proto_only") and self.ppnet.nearest_proto_only:
            l1_mask = 1 - torch.eye(self.ppnet.num_classes, device=image.device)
        else:
            l1_mask = 1 - torch.t(identity)
        l1 = (self.ppnet.last_layer.weight * l1_mask).norm(p=1)
        total = image.new_zeros((), dtype=torch.float32)
        ce_sum = kld_sum = None
        n_correct = torch.zeros((), dtype=torch.int64, device=image.device)
        n_patches = torch.zeros((), dtype=torch.int64, device=image.device)
        for logits, distances in outputs:
            B, h, w, K = logits.shape
            t = target
            if tuple(t.shape[-2:]) != (h, w):
                t = self.resize_fn(t.reshape(B, *t.shape[-2:]), h, w)
            target_img = t.reshape(B, -1).long()
            flat = target_img.reshape(-1)
            out = logits.reshape(-1, K)
            if self.ignore_void_class:  # module.py:156-160, without a host sync
                valid = flat != 0
                cls = torch.where(valid, flat - 1, torch.full_like(flat, -100))
            else:
                valid = torch.ones_like(flat, dtype=torch.bool)
                cls = flat
            ce = F.cross_entropy(out, cls, ignore_index=-100, reduction="sum")
            if self.loss_weight_kld != 0:
                kmean, npairs = self.kld_fn(distances, target_img, identity)
                knum = kmean * npairs.to(kmean.dtype)
            else:
                knum = npairs = torch.zeros((), device=image.device)
            counts = self._global(torch.stack([valid.sum().to(torch.float32),
                                               npairs.to(torch.float32).reshape(())]))
            n_ce = torch.clamp(counts[0], min=1.0)
            n_kld = counts[1]
            ce_term = ce / n_ce
            kld_term = torch.where(n_kld > 0, knum / torch.clamp(n_kld, min=1.0), torch.zeros_like(knum))
            loss = (self.loss_weight_crs_ent * ce_term + self.loss_weight_kld * kld_term +
                    self.loss_weight_l1 * l1 / world)
            total = total + loss / len(outputs)
            ce_sum = ce_term / len(outputs) if ce_sum is None else ce_sum + ce_term / len(outputs)
            kld_sum = kld_term / len(outputs) if kld_sum is None else kld_sum + kld_term / len(outputs)
            pred = torch.argmax(out, dim=-1)
            n_correct += ((pred == cls) & valid).sum()
            n_patches += valid.sum()
        return {"loss": total, "cross_entropy": ce_sum, "kld_loss": kld_sum, "l1": l1.detach(),
                "n_correct": n_correct, "n_patches": n_patches}

    def __call__(self, image: Tensor, target: Tensor) -> Dict[str, Tensor]:
        if self.iter_steps == 0:
            # in place, as the reference's optimizer.zero_grad() (module.py:122; torch 1.10's
            # default): the gradients stay views into the exchange buckets' buffers
            self.optimizer.zero_grad(set_to_none=False)
        boundary = self.iter_steps + 1 == self.iter_size
        if boundary:
            self.buckets.arm()  # the exchange rides on this backward's gradient hooks
        parts = self.loss(image, target)
        (parts["loss"] / self.iter_size).backward()
        self.iter_steps += 1
        if boundary:
            self.finish_accumulation()
        return {k: v.detach() for k, v in parts.items()}

    def finish_accumulation(self) -> None:
        """The accumulation boundary: gradient exchange (if not already overlapped), optimizer
        and scheduler step (module.py:238-243)."""
        self.buckets.wait()
        self.optimizer.step()
        if self.lr_scheduler is not None:
            self.lr_scheduler.step()
        self.iter_steps = 0
