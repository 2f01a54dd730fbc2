"""ORACLE — test infrastructure only. CPU restatement of the reference's push argmin core.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
Parity against the reference binary is UNPINNED (reference import denied, no reference
fixtures); see protoseg_oracle.py's header.

``update_prototypes_on_image_core`` restates segmentation/push.py:184-281 with the same
Python loops, the same float64 patch arithmetic int(pixel / (img_size / fmap_size)), the same
``set`` of (i, j) tuples turned into a list (so the same tie order as the reference under
CPython), the same np.argmin and the same strict '<' against float64 accumulators.
``class_patch_bitmask_fast`` is a vectorised equivalent of the per-pixel loop for large
inputs (checked against the loop on small ones).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np

# segmentation/constants.py:83-112 (raw Cityscapes id -> 0 = void, 1..19 = eval classes)
CITYSCAPES_19_EVAL_CATEGORIES = {
    0: 0, 1: 1, 2: 2, 3: 0, 4: 0, 5: 3, 6: 4, 7: 5, 8: 0, 9: 0, 10: 0, 11: 6, 12: 0, 13: 7, 14: 8,
    15: 9, 16: 10, 17: 11, 18: 12, 19: 13, 20: 14, 21: 15, 22: 16, 23: 0, 24: 0, 25: 17, 26: 18,
    27: 19, 28: 0,
}


def convert_targets(img_y: np.ndarray, mapping: Dict[int, int] = CITYSCAPES_19_EVAL_CATEGORIES) -> np.ndarray:
    """dataset.py:63-64: np.vectorize(MAPPING.get)"""
    return np.vectorize(mapping.get)(img_y)


def class_to_patch_index_dict(img_y: np.ndarray, h: int, w: int, num_classes: int) -> Dict[int, List[tuple]]:
    """push.py:195-230 (pure Python; a 1024x2048 label takes seconds)."""
    img_height, img_width = img_y.shape[0], img_y.shape[1]
    patch_height = img_height / h
    patch_width = img_width / w
    sets = {key: set() for key in range(num_classes)}
    for pixel_i in range(img_y.shape[0]):
        patch_i = int(pixel_i / patch_height)
        for pixel_j in range(img_y.shape[1]):
            patch_j = int(pixel_j / patch_width)
            pixel_cls = int(img_y[pixel_i, pixel_j])
            if pixel_cls > 0:
                sets[pixel_cls - 1].add((patch_i, patch_j))
    return {k: list(v) for k, v in sets.items()}


def class_to_patch_index_dict_torch(img_y, h: int, w: int, num_classes: int) -> Dict[int, List[tuple]]:
    """push.py:186 + 214-230 as the reference runs them: the label map as a torch.LongTensor and
    one `int(img_y[i, j].item())` per pixel (the CPU baseline's timed loop; same sets as
    class_to_patch_index_dict)."""
    import torch
    img_y = torch.LongTensor(np.asarray(img_y))
    patch_height = img_y.shape[0] / h
    patch_width = img_y.shape[1] / w
    sets = {key: set() for key in range(num_classes)}
    for pixel_i in range(img_y.shape[0]):
        patch_i = int(pixel_i / patch_height)
        for pixel_j in range(img_y.shape[1]):
            patch_j = int(pixel_j / patch_width)
            pixel_cls = int(img_y[pixel_i, pixel_j].item())
            if pixel_cls > 0:
                sets[pixel_cls - 1].add((patch_i, patch_j))
    return {k: list(v) for k, v in sets.items()}


def class_patch_bitmask_fast(img_y: np.ndarray, h: int, w: int) -> np.ndarray:
    """Vectorised class bitmask per patch, uint32 [h*w]: bit c-1 set iff a pixel of class c>0
    maps to the patch (same float64 division as push.py:217-219)."""
    H, W = img_y.shape
    pi = (np.arange(H, dtype=np.float64) / (H / h)).astype(np.int64)
    pj = (np.arange(W, dtype=np.float64) / (W / w)).astype(np.int64)
    cls = img_y.astype(np.int64)
    valid = (cls > 0) & (cls <= 32)
    bits = np.where(valid, np.left_shift(np.uint64(1), np.clip(cls - 1, 0, 63).astype(np.uint64)), 0).astype(np.uint64)
    patch = (pi[:, None] * w + pj[None, :]).reshape(-1)
    out = np.zeros(h * w, dtype=np.uint64)
    np.bitwise_or.at(out, patch, bits.reshape(-1))
    return out.astype(np.uint32)


def bitmask_from_dict(sets: Dict[int, List[tuple]], h: int, w: int) -> np.ndarray:
    out = np.zeros(h * w, dtype=np.uint32)
    for k, patches in sets.items():
        for (i, j) in patches:
            out[i * w + j] |= np.uint32(1 << k)
    return out


class PushOracleState:
    """push.py:55-81: float64 accumulators and receptive-field boxes."""

    def __init__(self, n_prototypes: int, depth: int, with_class: bool = True):
        self.global_min_proto_dist = np.full(n_prototypes, np.inf)
        self.global_min_fmap_patches = np.zeros([n_prototypes, depth, 1, 1])
        self.proto_rf_boxes = np.full(shape=[n_prototypes, 6 if with_class else 5], fill_value=-1)
        self.winner_patch = np.full(n_prototypes, -1, dtype=np.int64)  # (i*w + j), for comparisons


def update_prototypes_on_image_core(state: PushOracleState, protoL_input_: np.ndarray, proto_dist_: np.ndarray,
                                    img_y: np.ndarray, proto_class: Sequence[int], num_classes: int,
                                    start_index_of_search_batch: int,
                                    sets: Optional[Dict[int, List[tuple]]] = None) -> None:
    """push.py:195-307 (argmin core + rf boxes).

    protoL_input_: [C, h, w] float32 features; proto_dist_: [h, w, P] float32 distances
    (push.py:209-210); img_y: [H, W] class labels after convert_targets."""
    model_output_height, model_output_width = protoL_input_.shape[1], protoL_input_.shape[2]
    img_height, img_width = img_y.shape[0], img_y.shape[1]
    patch_height = img_height / model_output_height
    patch_width = img_width / model_output_width
    if sets is None:
        sets = class_to_patch_index_dict(img_y, model_output_height, model_output_width, num_classes)
    n_prototypes = proto_dist_.shape[2]
    for j in range(n_prototypes):
        target_class = int(proto_class[j])
        if len(sets[target_class]) == 0:
            continue
        all_dist = np.asarray([proto_dist_[patch_i, patch_j, j] for patch_i, patch_j in sets[target_class]])
        batch_argmin_proto_dist = np.argmin(all_dist)
        batch_min_proto_dist = all_dist[batch_argmin_proto_dist]
        if batch_min_proto_dist < state.global_min_proto_dist[j]:
            patch_i, patch_j = sets[target_class][batch_argmin_proto_dist]
            state.global_min_proto_dist[j] = batch_min_proto_dist
            state.global_min_fmap_patches[j] = protoL_input_[:, patch_i:patch_i + 1, patch_j:patch_j + 1]
            state.winner_patch[j] = patch_i * model_output_width + patch_j
            state.proto_rf_boxes[j, 0] = start_index_of_search_batch
            state.proto_rf_boxes[j, 1] = int(patch_i * patch_height)
            state.proto_rf_boxes[j, 2] = int(patch_i * patch_height + patch_height) + 1
            state.proto_rf_boxes[j, 3] = int(patch_j * patch_width)
            state.proto_rf_boxes[j, 4] = int(patch_j * patch_width + patch_width) + 1
            if state.proto_rf_boxes.shape[1] == 6:
                state.proto_rf_boxes[j, 5] = target_class


def masked_argmin_fast(proto_dist_: np.ndarray, bitmask: np.ndarray, proto_class: Sequence[int]):
    """Vectorised per-prototype masked min over one image: (min d [P] float32 or inf,
    lowest patch index attaining it [P] or -1, second-smallest distinct-patch d [P])."""
    h, w, P = proto_dist_.shape
    d = proto_dist_.reshape(h * w, P).astype(np.float32)
    cls = np.asarray(proto_class, dtype=np.int64)
    member = ((bitmask[:, None].astype(np.uint64) >> cls[None, :].astype(np.uint64)) & 1).astype(bool)
    dm = np.where(member, d, np.float32(np.inf))
    idx = np.argmin(dm, axis=0)
    best = dm[idx, np.arange(P)]
    idx = np.where(np.isinf(best), -1, idx)
    dm2 = dm.copy()
    dm2[np.maximum(idx, 0), np.arange(P)] = np.inf
    second = dm2.min(axis=0)
    return best, idx, second


def dedup(prototype_update: np.ndarray):
    """push.py:147-152 -> (unique_index, duplicate_idx)"""
    _, unique_index = np.unique(prototype_update, axis=0, return_index=True)
    duplicate_idx = [i for i in range(prototype_update.shape[0]) if i not in unique_index]
    return unique_index, duplicate_idx
