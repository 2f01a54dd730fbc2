"""ORACLE — test infrastructure only. CPU restatement of the reference's mIoU evaluation.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline; the product path never calls it.

Restates segmentation/eval_valid.py:159-219 per image (torch CPU, float32):
  logits NHWC -> permute(0, 3, 1, 2) (161) -> F.interpolate(size=ann.shape, bilinear,
  align_corners=False) (171) -> argmax over classes (176);
  distances -> the same interpolation (172) -> argmin over prototypes (174);
  correct += sum(((pred + 1) == ann) & (ann != 0)); total += sum(ann != 0) (178-180);
  per class c: I[c] += sum(pred == c & ann == c + 1); U[c] += sum((pred == c | ann == c + 1) & ann != 0)
  (182-189); per prototype p of class k: pixels whose nearest prototype is p and pred == k
  (191-197); pixel accuracy and mIoU (216-219).
The random-pixel top-k statistic (200-214) draws from np.random without a seed in the reference
and is not restated.

Parity status: UNPINNED against the reference itself (import denied; no reference
tests). The bilinear weights follow torch's align_corners=False source index.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F


def eval_counts(logits_nhwc: torch.Tensor, anns: np.ndarray, K: int, distances: Optional[torch.Tensor] = None,
                proto_class: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
    """logits_nhwc [B, h, w, K]; anns [B, H, W] int (already CLS_CONVERT-ed, 0 = void);
    distances [B, P, h, w] (optional); proto_class [P]."""
    batch_logits = logits_nhwc.permute(0, 3, 1, 2)                                      # eval_valid.py:161
    correct = total = 0
    I = np.zeros(K, np.int64)
    U = np.zeros(K, np.int64)
    pc = np.zeros(0 if distances is None else distances.shape[1], np.int64)
    for sample_i in range(batch_logits.shape[0]):                                       # eval_valid.py:166
        ann = anns[sample_i]
        logits = torch.unsqueeze(batch_logits[sample_i], 0)
        logits = F.interpolate(logits, size=ann.shape, mode="bilinear", align_corners=False)[0]   # 171
        pred = torch.argmax(logits, dim=0).numpy()                                      # eval_valid.py:176
        correct += int(np.sum(((pred + 1) == ann) & (ann != 0)))                        # eval_valid.py:178
        total += int(np.sum(ann != 0))                                                  # eval_valid.py:180
        for cls_i in range(K):                                                          # eval_valid.py:182-189
            pr = pred == cls_i
            gt = ann == cls_i + 1
            I[cls_i] += int(np.sum(pr & gt))
            U[cls_i] += int(np.sum((pr | gt) & (ann != 0)))
        if distances is not None:
            d = torch.unsqueeze(distances[sample_i], 0)
            d = F.interpolate(d, size=ann.shape, mode="bilinear", align_corners=False)[0]   # eval_valid.py:172
            nearest_proto = torch.argmin(d, dim=0).numpy()                             # eval_valid.py:174
            nearest_cls = proto_class[nearest_proto]                                    # PROTO2CLS, :192
            for class_i in range(K):                                                    # eval_valid.py:194-197
                is_class_proto = (pred == class_i) & (nearest_cls == class_i)
                for proto_num in np.nonzero(proto_class == class_i)[0]:
                    pc[proto_num] += int(np.sum(is_class_proto & (nearest_proto == proto_num)))
    return {"correct": np.int64(correct), "total": np.int64(total), "I": I, "U": U, "proto_counts": pc}


def metrics(correct, total, I, U):
    """eval_valid.py:216-219: pixel accuracy and mIoU over classes with a non-empty union."""
    pixel_accuracy = correct / total * 100
    cls_iou = {c: (I[c] * 100) / u for c, u in enumerate(U) if u > 0}
    return float(pixel_accuracy), float(np.mean(list(cls_iou.values()))), cls_iou


def interpolated_margins(logits_nhwc: torch.Tensor, size) -> torch.Tensor:
    """float64 bilinear logits at full size and the top-1 minus top-2 margin per pixel (tests use
    it to separate genuinely decided pixels from near-ties)."""
    up = F.interpolate(logits_nhwc.permute(0, 3, 1, 2).double(), size=size, mode="bilinear", align_corners=False)
    top2 = torch.topk(up, 2, dim=1).values
    return top2[:, 0] - top2[:, 1]
