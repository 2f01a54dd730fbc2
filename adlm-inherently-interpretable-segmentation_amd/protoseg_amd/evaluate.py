"""Segmentation evaluation (segmentation/eval_valid.py:131-219) on the HIP counting kernel.

The reference upsamples each image's logits and distances to the label resolution, takes
argmax / argmin and counts on the host with numpy; ``SegmentationEvaluator.update`` does the
same counting in one kernel per batch (``protoseg_eval_counts``) without materialising the
upsampled tensors, and ``result()`` applies the reference's formulas (eval_valid.py:216-219).
The random-pixel top-k statistic (eval_valid.py:200-214, unseeded np.random) is not produced.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
from torch import Tensor

from . import _lib

_LABEL_DTYPES = {torch.int64: _lib.I64, torch.int32: _lib.I32, torch.uint8: _lib.U8}


def eval_counts(logits: Tensor, anns: Tensor, counts: Tensor, distances: Optional[Tensor] = None,
                proto_class: Optional[Tensor] = None, lut: Optional[Tensor] = None) -> Tensor:
    """Adds one batch to ``counts`` (int64 [2 + 2K (+ P)]): correct, total, I[K], U[K] and, with
    distances, the per-prototype counts. logits [B, h, w, K] (NHWC, PPNet.forward), anns [B, H, W]
    labels (0 = void; raw ids when ``lut`` maps them), distances [B, P, h, w]."""
    dev = _lib.require_device(logits, anns, counts, distances, proto_class, lut)
    lg = logits.float().contiguous()
    B, h, w, K = lg.shape
    a = anns if anns.dtype in _LABEL_DTYPES else anns.to(torch.int64)
    a = a.contiguous()
    H, W = a.shape[-2:]
    d = distances.float().contiguous() if distances is not None else None
    P = d.shape[1] if d is not None else 0
    pc = proto_class.to(torch.int32).contiguous() if proto_class is not None else None
    lt = lut.to(torch.int32).contiguous() if lut is not None else None
    if counts.dtype != torch.int64 or counts.numel() < 2 + 2 * K + P:
        raise _lib.ProtosegError(f"counts must be int64 with >= {2 + 2 * K + P} elements")
    with torch.cuda.device(dev):
        _lib.call("protoseg_eval_counts", _lib.ptr(lg), _lib.ptr(d), B, h, w, K, P, _lib.ptr(a), _LABEL_DTYPES[a.dtype],
                  H, W, _lib.ptr(lt), 0 if lt is None else lt.numel(), _lib.ptr(pc), _lib.ptr(counts),
                  _lib.stream_of(dev))
    return counts


class SegmentationEvaluator:
    """Accumulates eval_valid.py's counters over batches: correct/total pixels, CLS_I / CLS_U per
    class, and cls_prototype_counts per prototype (eval_valid.py:120-197)."""

    def __init__(self, num_classes: int, proto_class: Optional[Tensor] = None, device="cuda"):
        self.K = num_classes
        self.proto_class = proto_class.to(device) if proto_class is not None else None
        P = 0 if proto_class is None else proto_class.numel()
        self.counts = torch.zeros(2 + 2 * num_classes + P, dtype=torch.int64, device=device)

    def update(self, logits: Tensor, anns: Tensor, distances: Optional[Tensor] = None,
               lut: Optional[Tensor] = None) -> None:
        eval_counts(logits, anns, self.counts, distances if self.proto_class is not None else None,
                    self.proto_class, lut)

    def result(self) -> Dict[str, object]:
        c = self.counts.cpu().numpy()
        K = self.K
        correct, total, I, U = int(c[0]), int(c[1]), c[2:2 + K], c[2 + K:2 + 2 * K]
        cls_iou = {k: float(I[k] * 100) / float(u) for k, u in enumerate(U) if u > 0}   # eval_valid.py:218
        return {"pixel_accuracy": correct / total * 100 if total else float("nan"),    # eval_valid.py:216
                "mean_iou": float(np.mean(list(cls_iou.values()))) if cls_iou else float("nan"),  # :219
                "class_iou": cls_iou, "correct": correct, "total": total, "I": I, "U": U,
                "prototype_counts": c[2 + 2 * K:]}
