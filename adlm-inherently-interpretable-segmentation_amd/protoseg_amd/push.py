"""Prototype push (nearest-patch projection) on the HIP kernels.

Mirrors reference segmentation/push.py:24-158 (``push_prototypes``) and the argmin core of
162-280 (``update_prototypes_on_image``). The reference copies every image's distance map to
the host and runs a 2M-iteration Python loop per image plus a per-prototype gather and
np.argmin; here the label->patch mask, the fused distance + masked argmin and the strict-'<'
merge all run on the device, and the host only touches P-sized results at the end.

Semantics kept from the reference:
  * patch of pixel (i, j) = (int(i / (H / h)), int(j / (W / w))) in float64 (push.py:201-223);
  * class c > 0 marks class index c-1 (push.py:222-223); prototypes of a class absent from
    the image are skipped (push.py:255-256);
  * a prototype moves only on a strictly smaller distance; images are visited in
    ``dataset.img_ids`` order, so an earlier image wins a tie (push.py:101, 265);
  * receptive-field boxes push.py:288-307, dedup push.py:147-155, prune model.py:311-336;
  * high-activation bound boxes push.py:309-343 + helpers.py:48-82 (bbox.hip), computed once
    per prototype on its final winning image — the reference recomputes them on every image
    that improves the prototype and keeps the last, i.e. the same image.
  * exact ties between patches of ONE image resolve in the reference's order: the kernel
    takes the lowest patch index and flags the tie (runner-up distance == minimum); the host
    then redoes np.argmin over the class patches in the list(set) order of push.py:214-230
    for those prototypes only (``resolve_exact_ties``).

Out of scope (host-side visualisation, needs cv2/matplotlib): the PNG outputs of
push.py:344-481.
"""
from __future__ import annotations

import json
import math
import weakref
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
from torch import Tensor

from . import _lib

# segmentation/constants.py:6-7 (ImageNet statistics used by to_normalized_tensor)
CITYSCAPES_MEAN = (0.485, 0.456, 0.406)
CITYSCAPES_STD = (0.229, 0.224, 0.225)


def _label_dtype(t: Tensor) -> int:
    return {torch.int64: _lib.I64, torch.int32: _lib.I32, torch.uint8: _lib.U8}.get(t.dtype, -1)


def mask_words(num_classes: int) -> int:
    """32-bit class-mask planes for ``num_classes`` classes (classes 0 .. K-1 = labels 1 .. K)."""
    return max(1, (int(num_classes) + 31) // 32)


def patch_class_mask(labels: Tensor, h: int, w: int, lut: Optional[Tensor] = None, words: int = 1) -> Tensor:
    """labels [n, H, W] (int64 / int32 / uint8, device) -> int32 [n, h*w] holding the uint32
    class bitmask of each patch (bit k <=> a pixel of class k+1). ``lut`` [L] int32 maps raw
    label ids first (CITYSCAPES_19_EVAL_CATEGORIES / PASCAL_ID_MAPPING as a table). More than 32
    classes: ``words`` planes, int32 [words, n, h*w] (plane q: classes 32q+1 .. 32q+32)."""
    dev = _lib.require_device(labels, lut)
    if labels.dim() == 2:
        labels = labels.unsqueeze(0)
    labels = labels.contiguous()
    dt = _label_dtype(labels)
    if dt < 0:
        raise _lib.ProtosegError(f"label dtype {labels.dtype} unsupported (int64, int32, uint8)")
    n, H, W = labels.shape
    mask = torch.empty((n, h * w) if words == 1 else (words, n, h * w), device=dev, dtype=torch.int32)
    lut_c = lut.to(torch.int32).contiguous() if lut is not None else None
    with torch.cuda.device(dev):
        _lib.call("protoseg_patch_class_mask_words", _lib.ptr(labels), dt, n, H, W, h, w, _lib.ptr(lut_c),
                  0 if lut_c is None else lut_c.numel(), int(words), _lib.ptr(mask), _lib.stream_of(dev))
    return mask


def push_argmin(x: Tensor, protos: Tensor, proto_class: Tensor, mask: Tensor, with_second: bool = False):
    """Per image and prototype, the masked minimum key (float_bits(d) << 32 | patch) as int64
    storage of uint64 [n, P]; -1 (all ones) when the image has no patch of the class. With
    ``with_second`` also the runner-up of the same image (float_bits(d2) << 32 | 0xFFFFFFFF: the
    second-smallest class-patch distance), as a pair. A [words, n, h*w] mask (more than 32
    classes) takes the wide path (protoseg_push_argmin_words)."""
    dev = _lib.require_device(x, protos, proto_class, mask)
    words = 1 if mask.dim() == 2 else int(mask.shape[0])
    x = x.float().contiguous()
    protos = protos.reshape(protos.shape[0], -1).float().contiguous()
    n, C, h, w = x.shape
    P = protos.shape[0]
    if protos.shape[1] != C:
        raise _lib.ProtosegError(f"push_argmin: prototypes hold {protos.shape[1]} values, the map {C} channels")
    keys = torch.empty((n, P), device=dev, dtype=torch.int64)
    second = torch.empty_like(keys) if with_second else None
    with torch.cuda.device(dev):
        _lib.call("protoseg_push_argmin_words", _lib.ptr(x), n, C, h, w, _lib.ptr(protos), P,
                  _lib.ptr(proto_class.to(torch.int32).contiguous()), _lib.ptr(mask.contiguous()), words,
                  _lib.ptr(keys), _lib.ptr(second), _lib.stream_of(dev))
    return (keys, second) if with_second else keys


def decode_keys(keys: Tensor):
    """int64-stored uint64 keys -> (dist float32, patch int64, found bool)."""
    k = keys.to(torch.int64)
    found = k != -1
    hi = ((k >> 32) & 0xFFFFFFFF).to(torch.int32)
    dist = hi.view(torch.float32) if hi.is_contiguous() else hi.contiguous().view(torch.float32)
    return dist, (k & 0xFFFFFFFF), found


@dataclass
class PushState:
    """Running global minimum (push.py:55-61): distance, image index, patch index, feature
    vector; plus the runner-up distance over every class patch seen (near-tie flags)."""
    dist: Tensor
    img: Tensor
    patch: Tensor
    fmap: Tensor
    second: Optional[Tensor] = None
    near_ties: Optional[np.ndarray] = None
    # per image index: (H_img, W_img, h, w) needed for the receptive-field boxes
    geometry: Dict[int, tuple] = field(default_factory=dict)

    @classmethod
    def create(cls, P: int, C: int, device) -> "PushState":
        return cls(dist=torch.full((P,), math.inf, device=device, dtype=torch.float32),
                   img=torch.full((P,), -1, device=device, dtype=torch.int64),
                   patch=torch.full((P,), -1, device=device, dtype=torch.int32),
                   fmap=torch.zeros((P, C), device=device, dtype=torch.float32),
                   second=torch.full((P,), math.inf, device=device, dtype=torch.float32))


_words_cache: Dict[tuple, tuple] = {}


def _class_words(proto_class: Tensor) -> int:
    """mask_words(max class + 1), cached per (tensor, version): reading the maximum of a device
    tensor is a device -> host sync, paid once per prototype-class tensor, not once per batch."""
    key = (id(proto_class), proto_class.data_ptr(), proto_class._version, proto_class.numel(), str(proto_class.device))
    hit = _words_cache.get(key)
    if hit is not None and hit[0]() is proto_class:  # not a new tensor reusing a freed one's id / address
        return hit[1]
    if len(_words_cache) > 64:
        _words_cache.clear()
    w = mask_words(int(proto_class.max()) + 1)
    _words_cache[key] = (weakref.ref(proto_class), w)
    return w


def push_update(state: PushState, x: Tensor, labels: Tensor, protos: Tensor, proto_class: Tensor, first_img: int,
                lut: Optional[Tensor] = None, words: Optional[int] = None) -> None:
    """One batch of images (dataset indices first_img ..): mask -> argmin -> strict-'<' merge.
    This is push_prototypes' inner step (one call per batch of equal-geometry images)."""
    x = x.float().contiguous()
    n, C, h, w = x.shape
    if labels.dim() == 2:
        labels = labels.unsqueeze(0)
    labels = labels.contiguous()
    dt = _label_dtype(labels)
    if dt < 0:
        raise _lib.ProtosegError(f"label dtype {labels.dtype} unsupported (int64, int32, uint8)")
    if words is None:  # class-mask planes (one below 33 classes); callers in a loop pass it
        words = _class_words(proto_class)
    dev = _lib.require_device(x, labels, protos, proto_class, lut)
    protos = protos.reshape(protos.shape[0], -1).float().contiguous()
    P = protos.shape[0]
    if protos.shape[1] != C:
        raise _lib.ProtosegError(f"push projects 1x1 prototypes (depth {C}); got {protos.shape[1]} values per "
                                 "prototype (k x k prototypes: push.py's patch windows are not built here)")
    if state.second is None:
        state.second = torch.full((P,), math.inf, device=dev, dtype=torch.float32)
    pc = proto_class if proto_class.dtype == torch.int32 and proto_class.is_contiguous() \
        else proto_class.to(torch.int32).contiguous()
    lut_c = lut.to(torch.int32).contiguous() if lut is not None else None
    H, W = labels.shape[-2:]
    # mask -> top-2 argmin -> merge in one library call (masks and keys in its stream scratch)
    with torch.cuda.device(dev):
        _lib.call("protoseg_push_update", _lib.ptr(labels), dt, n, int(H), int(W), _lib.ptr(lut_c),
                  0 if lut_c is None else lut_c.numel(), int(words), _lib.ptr(x), C, h, w, _lib.ptr(protos), P,
                  _lib.ptr(pc), int(first_img), _lib.ptr(state.dist), _lib.ptr(state.second), _lib.ptr(state.img),
                  _lib.ptr(state.patch), _lib.ptr(state.fmap), _lib.stream_of(dev))
    for i in range(n):
        state.geometry[first_img + i] = (int(H), int(W), int(h), int(w))


def push_distances(x: Tensor, protos: Tensor, words: int = 1) -> Tensor:
    """Distances [m, h*w] of ``protos`` [m, C] at every patch of ONE image x [1, C, h, w] (or
    [C, h, w]) in push_argmin's arithmetic for a ``words``-plane mask, operation for operation: a
    tie here is exactly a tie that kernel saw."""
    dev = _lib.require_device(x, protos)
    x = x.float().contiguous()
    if x.dim() == 4:
        if x.shape[0] != 1:
            raise ValueError("push_distances takes one image")
        x = x[0]
    C, h, w = x.shape
    protos = protos.reshape(protos.shape[0], -1).float().contiguous()
    m = protos.shape[0]
    out = torch.empty((m, h * w), device=dev, dtype=torch.float32)
    with torch.cuda.device(dev):
        _lib.call("protoseg_push_distances_words", _lib.ptr(x), C, h, w, _lib.ptr(protos), m, int(words),
                  _lib.ptr(out), _lib.stream_of(dev))
    return out


def reference_patch_order(labels: np.ndarray, cls: int, h: int, w: int) -> List[tuple]:
    """``list(class_to_patch_index_dict[cls])`` of push.py:214-230: the patches of class ``cls``
    (label value cls + 1) in the iteration order of the Python set the reference builds. A set's
    order depends only on the sequence of first insertions, which is the row-major order of each
    patch's first pixel of the class (push.py:216-223 walk the pixels row by row), so the set is
    rebuilt here from that sequence: CPython's int-tuple hash is unseeded, and the reference's
    Python (3.9, env.yml:17) shares the tuple hash and set growth rule of this interpreter."""
    H, W = labels.shape
    patch_height, patch_width = H / h, W / w  # float64, push.py:201-202
    pix = np.flatnonzero(labels.reshape(-1) == cls + 1)
    if pix.size == 0:
        return []
    pi = (pix // W / patch_height).astype(np.int64)  # int(pixel_i / patch_height), push.py:217
    pj = (pix % W / patch_width).astype(np.int64)    # int(pixel_j / patch_width), push.py:219
    q = pi * w + pj
    uniq, first = np.unique(q, return_index=True)
    s = set()
    for patch in uniq[np.argsort(first, kind="stable")].tolist():
        s.add((patch // w, patch % w))
    return list(s)


def exact_tie_candidates(state: PushState) -> np.ndarray:
    """Prototypes whose winning distance equals the runner-up's exactly (the runner-up of the
    winning image, or an equal distance in a later image): only these can hold an exact tie
    inside their winning image, where the kernel's lowest-patch pick may differ from the
    reference's set order."""
    if state.second is None:
        return np.zeros(0, dtype=np.int64)
    tie = (state.img >= 0) & (state.second == state.dist)
    return np.nonzero(tie.cpu().numpy())[0]


def resolve_exact_ties(state: PushState, load: Callable, protos: Tensor, proto_class, lut: Optional[Tensor] = None,
                       candidates=None, log: Callable = print) -> List[int]:
    """push.py:249-263 in the reference's own order for the prototypes whose winning image holds
    several class patches at exactly the minimum distance: np.argmin over the class's patches in
    list(set) order picks the first of them (the kernel picked the lowest patch index).
    ``load(img_index)`` returns (x [1, C, h, w], labels [H, W]) of that image as the scan saw
    them. Updates state.patch / state.fmap in place; returns the prototypes that moved."""
    cand = exact_tie_candidates(state) if candidates is None else np.asarray(candidates, dtype=np.int64)
    if cand.size == 0:
        return []
    img = state.img.cpu().numpy()
    dist = state.dist.cpu().numpy()
    patch = state.patch.cpu().numpy()
    pcls = np.asarray(proto_class.cpu() if isinstance(proto_class, Tensor) else proto_class).astype(np.int64)
    lut_np = lut.cpu().numpy() if lut is not None else None
    pv = protos.detach().reshape(protos.shape[0], -1).float()
    words = mask_words(int(pcls.max()) + 1)  # the scan's mask planes, hence its arithmetic
    moved = []
    for im in np.unique(img[cand]):
        ids = cand[img[cand] == im]
        x, labels = load(int(im))
        x = x.float()
        _, C, h, w = x.shape
        lab = labels.reshape(labels.shape[-2:]).cpu().numpy().astype(np.int64)
        if lut_np is not None:  # the scan's table (dataset.convert_targets); ids outside it: no class
            ok = (lab >= 0) & (lab < lut_np.size)
            lab = np.where(ok, lut_np[np.clip(lab, 0, lut_np.size - 1)], -1)
        d = push_distances(x, pv[torch.as_tensor(ids, device=pv.device)], words).cpu().numpy()
        for k, j in enumerate(ids.tolist()):
            order = reference_patch_order(lab, int(pcls[j]), h, w)
            if not order:
                continue
            all_dist = d[k, [pi * w + pj for pi, pj in order]]
            q = int(np.argmin(all_dist))
            if all_dist[q] != dist[j]:
                log(f"\tprototype {j}: distances of image {im} not reproduced (tie left to the kernel)")
                continue
            pi, pj = order[q]
            if pi * w + pj != patch[j]:
                state.patch[j] = pi * w + pj
                state.fmap[j] = x[0, :, pi, pj].to(state.fmap.device)
                moved.append(j)
    return moved


def near_ties(state: PushState, protos: Tensor, rtol: float = 1e-5) -> np.ndarray:
    """Prototypes whose winning patch beats the runner-up (any image, any class patch) by no
    more than the f32 rounding band of the expanded distance, rtol * (||x||^2 + ||p||^2) with x
    the winning feature vector: there the reference's own rounding may pick the other patch
    (hard part 2); exact ties are resolved in the reference's order by
    ``resolve_exact_ties``. ``protos`` are the prototype vectors the push measured against."""
    if state.second is None:
        raise ValueError("push state has no runner-up distances")
    p = protos.detach().reshape(protos.shape[0], -1).float().to(state.fmap.device)
    band = rtol * ((state.fmap * state.fmap).sum(1) + (p * p).sum(1))
    found = state.img >= 0
    tie = found & torch.isfinite(state.second) & (state.second - state.dist <= band)
    return np.nonzero(tie.cpu().numpy())[0]


_ACT_KINDS = {"log": _lib.ACT_LOG, "linear": _lib.ACT_LINEAR, "identity": _lib.ACT_IDENTITY}


def act_upsample(dist: Tensor, H: int, W: int, act: str = "log", eps: float = 1e-4, max_dist: float = 0.0):
    """push.py:309-319: activation of each [h, w] distance map, then cv2.resize INTER_CUBIC to
    (H, W). ``dist`` [m, h, w] f32 on the device; returns (act [m, h, w], up [m, H, W])."""
    _lib.require_device(dist)
    if dist.dim() == 2:
        dist = dist.unsqueeze(0)
    dist = dist.float().contiguous()
    m, h, w = dist.shape
    if act not in _ACT_KINDS:
        raise ValueError(f"act {act!r}: one of {sorted(_ACT_KINDS)}")
    act_t = torch.empty_like(dist)
    up = torch.empty((m, int(H), int(W)), device=dist.device, dtype=torch.float32)
    with torch.cuda.device(dist.device):
        _lib.call("protoseg_act_upsample", _lib.ptr(dist), m, h, w, int(H), int(W), _ACT_KINDS[act], float(eps),
                  float(max_dist), _lib.ptr(act_t), _lib.ptr(up), _lib.stream_of(dist.device))
    return act_t, up


def bound_boxes(up: Tensor, labels: Tensor, target_class: Tensor, rf: Tensor, label_index: Optional[Tensor] = None,
                lut: Optional[Tensor] = None, percentile: float = 95.0, margin: int = 5):
    """push.py:321-343 + helpers.py:48-82 on the device. ``up`` [m, H, W] f32; ``labels``
    [n, H, W] (or [H, W]) int64/int32/uint8; ``target_class`` [m]; ``rf`` [m, 4] =
    (start_h, end_h, start_w, end_w). Returns (threshold [m] f32, box [m, 4] int32)."""
    _lib.require_device(up, labels, target_class, rf, label_index, lut)
    if labels.dim() == 2:
        labels = labels.unsqueeze(0)
    labels = labels.contiguous()
    dt = _label_dtype(labels)
    if dt < 0:
        labels, dt = labels.to(torch.int64), _lib.I64
    m, H, W = up.shape
    if tuple(labels.shape[1:]) != (H, W):
        raise ValueError(f"labels {tuple(labels.shape)} do not match maps {tuple(up.shape)}")
    tc = target_class.to(torch.int32).contiguous()
    rf32 = rf.to(torch.int32).contiguous()
    li = label_index.to(torch.int32).contiguous() if label_index is not None else None
    lut32 = lut.to(torch.int32).contiguous() if lut is not None else None
    if tc.numel() != m or rf32.shape != (m, 4) or (li is not None and li.numel() != m):
        raise ValueError("target_class [m], rf [m, 4] and label_index [m] must match up [m, H, W]")
    thr = torch.empty(m, device=up.device, dtype=torch.float32)
    box = torch.empty((m, 4), device=up.device, dtype=torch.int32)
    with torch.cuda.device(up.device):
        _lib.call("protoseg_bound_boxes", _lib.ptr(up.contiguous()), m, H, W, _lib.ptr(labels), dt, labels.shape[0],
                  _lib.ptr(li), _lib.ptr(lut32), 0 if lut32 is None else lut32.numel(), _lib.ptr(tc), _lib.ptr(rf32),
                  float(percentile), int(margin), _lib.ptr(thr), _lib.ptr(box), _lib.stream_of(up.device))
    return thr, box


def batch_bound_boxes(items, protos: Tensor, proto_class: np.ndarray, rf_boxes_all: np.ndarray, act: str = "log",
                      eps: float = 1e-4, act_fn: Optional[Callable] = None, lut: Optional[Tensor] = None):
    """Bound boxes (push.py:309-343) of every pushed prototype in one act_upsample + one
    bound_boxes launch per image geometry. ``items`` yields (proto_ids, x [1, C, h, w],
    labels [H, W]) per winning image. Returns {prototype id: (start_h, end_h, start_w, end_w)}."""
    from .ops import l2_distances, max_protos
    groups: Dict[tuple, dict] = {}
    for ids, x, labels in items:
        idt = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=x.device)
        # f32 distances (the push's own arithmetic); more winners on one image than one f32
        # call holds (P > 384 at C = 64, e.g. 30 prototypes/class) go in slices
        step = max_protos(x.shape[1], "f32")
        if step <= 0:
            raise _lib.ProtosegError(f"no f32 layer kernel for C={x.shape[1]}")
        pv = protos.detach()
        dist = torch.cat([l2_distances(x.float(), pv[idt[s:s + step]], eps, precision="f32")[0]
                          for s in range(0, len(idt), step)], 0)  # [m_i, h, w]
        key = (tuple(dist.shape[1:]), tuple(labels.shape[-2:]), labels.dtype)
        g = groups.setdefault(key, {"ids": [], "dist": [], "labels": [], "li": []})
        g["li"].extend([len(g["labels"])] * len(ids))
        g["ids"].extend(int(j) for j in ids)
        g["dist"].append(dist)
        g["labels"].append(labels.reshape(labels.shape[-2:]))
    max_dist = float(np.prod(protos.shape[1:]))  # push.py:229 prototype_shape[1] * [2] * [3]
    out: Dict[int, tuple] = {}
    for (_, (H, W), _), g in groups.items():
        dist = torch.cat(g["dist"], 0)
        kind = act
        if kind not in ("log", "linear"):
            if act_fn is None:
                raise ValueError(f"activation {act!r} needs prototype_activation_function_in_numpy")
            dist = torch.as_tensor(np.ascontiguousarray(act_fn(dist.cpu().numpy())), dtype=torch.float32,
                                   device=dist.device)
            kind = "identity"
        _, up = act_upsample(dist, H, W, kind, eps, max_dist)
        ids = np.asarray(g["ids"])
        dev = dist.device
        tc = torch.as_tensor(np.asarray(proto_class, dtype=np.int32)[ids], device=dev)
        rf = torch.as_tensor(np.asarray(rf_boxes_all)[ids, 1:5].astype(np.int32), device=dev)
        li = torch.as_tensor(np.asarray(g["li"], dtype=np.int32), device=dev)
        _, box = bound_boxes(up, torch.stack(g["labels"], 0), tc, rf, li, lut=lut)
        del up
        for j, b in zip(ids, box.cpu().numpy().astype(np.int64)):
            out[int(j)] = tuple(int(v) for v in b)
    return out


def prototype_classes(ppnet) -> Tensor:
    """push.py:251: target_class = argmax(prototype_class_identity[j])."""
    return torch.argmax(ppnet.prototype_class_identity, dim=1).to(torch.int32)


def rf_boxes(state: PushState, proto_class: np.ndarray, with_class: bool = True) -> np.ndarray:
    """push.py:288-307: [img, h_start, h_end, w_start, w_end(, class)] in float64 arithmetic."""
    img = state.img.cpu().numpy()
    patch = state.patch.cpu().numpy()
    P = img.shape[0]
    boxes = np.full((P, 6 if with_class else 5), -1, dtype=np.int64)
    for j in range(P):
        if img[j] < 0:
            continue
        H, W, h, w = state.geometry[int(img[j])]
        patch_height, patch_width = H / h, W / w
        patch_i, patch_j = divmod(int(patch[j]), w)
        boxes[j, 0] = img[j]
        boxes[j, 1] = int(patch_i * patch_height)
        boxes[j, 2] = int(patch_i * patch_height + patch_height) + 1
        boxes[j, 3] = int(patch_j * patch_width)
        boxes[j, 4] = int(patch_j * patch_width + patch_width) + 1
        if with_class:
            boxes[j, 5] = proto_class[j]
    return boxes


def lut_from_convert_targets(convert_targets) -> Optional[np.ndarray]:
    """Turns the reference's ``np.vectorize(MAPPING.get)`` (dataset.py:63-69) into a table."""
    fn = getattr(convert_targets, "pyfunc", convert_targets)
    mapping = getattr(fn, "__self__", None)
    if not isinstance(mapping, dict) or not mapping:
        return None
    keys = [k for k in mapping if isinstance(k, (int, np.integer))]
    if len(keys) != len(mapping) or min(keys) < 0:
        return None
    lut = np.full(max(keys) + 1, -1, dtype=np.int32)
    for k, v in mapping.items():
        lut[k] = v
    return lut


def to_normalized_tensor(img, mean=CITYSCAPES_MEAN, std=CITYSCAPES_STD) -> Tensor:
    """find_nearest.py:21-24: ToTensor (uint8 HWC -> float CHW / 255) then Normalize."""
    arr = np.asarray(img, dtype=np.uint8)
    t = torch.from_numpy(arr.copy()).permute(2, 0, 1).float().div(255.0)
    m = torch.tensor(mean, dtype=torch.float32).view(-1, 1, 1)
    s = torch.tensor(std, dtype=torch.float32).view(-1, 1, 1)
    return (t - m) / s


def dedup_and_prune(ppnet, fmap: np.ndarray, root_dir: Optional[str], log: Callable = print) -> List[int]:
    """push.py:143-155: write prototypes, np.unique(axis=0) dedup, prune, unique_prototypes.json."""
    shape = tuple(ppnet.prototype_shape)
    update = np.reshape(fmap.astype(np.float64), shape)
    with torch.no_grad():  # (a tracked in-place write: Adam.operands_ready sees the version move)
        ppnet.prototype_vectors.copy_(torch.tensor(update, dtype=torch.float32).to(ppnet.prototype_vectors.device))
    _, unique_index = np.unique(update, axis=0, return_index=True)
    unique_set = set(int(i) for i in unique_index)
    duplicate_idx = [i for i in range(ppnet.num_prototypes) if i not in unique_set]
    log(f"Removing {len(duplicate_idx)} duplicate prototypes.")
    ppnet.prune_prototypes(duplicate_idx)
    if root_dir is not None:
        os.makedirs(root_dir, exist_ok=True)
        with open(os.path.join(root_dir, "unique_prototypes.json"), "w") as fp:
            json.dump([int(i) for i in sorted(unique_index)], fp)
    return duplicate_idx


def push_prototypes(dataset, prototype_network_parallel, prototype_layer_stride=1,
                    root_dir_for_saving_prototypes=None, epoch_number=None, prototype_img_filename_prefix=None,
                    prototype_self_act_filename_prefix=None, proto_bound_boxes_filename_prefix=None,
                    save_prototype_class_identity=True, log=print, pascal=False,
                    prototype_activation_function_in_numpy=None, images_per_batch: int = 8,
                    process_group=None):
    """Drop-in for segmentation/push.py:24-158 (same arguments and side effects, minus the
    visualisation PNGs). With torch.distributed initialised (or ``process_group`` given) and
    world size > 1, every rank scans a contiguous shard of ``dataset.img_ids`` and the shards
    are merged exactly (distributed.reduce_push_state): the result equals the serial scan."""
    from PIL import Image

    from .distributed import reduce_bound_boxes, reduce_push_state, shard_bounds, world_info

    ppnet = prototype_network_parallel.module if hasattr(prototype_network_parallel, "module") \
        else prototype_network_parallel
    ppnet.eval()
    log("\tpush")
    start = time.time()
    device = ppnet.prototype_vectors.device
    P = ppnet.num_prototypes
    shape = tuple(ppnet.prototype_shape)
    kh, kw = (shape[2], shape[3]) if len(shape) == 4 else (1, 1)
    C = int(np.prod(shape[1:]))  # values per prototype: the k x k window, C k k deep

    def scan_features(f):
        """The push's view of a feature map: each k x k window as one column (push.py:276-280
        takes protoL_input_[:, i:i+h, j:j+w]), the 1 x 1 kernels on a C k k deep map."""
        if (kh, kw) == (1, 1):
            return f
        n, c, H, W = f.shape
        return torch.nn.functional.unfold(f, (kh, kw)).reshape(n, c * kh * kw, H - kh + 1, W - kw + 1)

    proto_class_t = prototype_classes(ppnet).to(device)
    proto_class = proto_class_t.cpu().numpy()
    words = mask_words(int(proto_class.max()) + 1)
    state = PushState.create(P, C, device)

    proto_epoch_dir = None
    if root_dir_for_saving_prototypes is not None:
        proto_epoch_dir = (os.path.join(root_dir_for_saving_prototypes, f"epoch-{epoch_number}")
                           if epoch_number is not None else root_dir_for_saving_prototypes)
        os.makedirs(proto_epoch_dir, exist_ok=True)
    if prototype_img_filename_prefix is not None or prototype_self_act_filename_prefix is not None:
        log("\tprototype visualisation PNGs are not produced by this build (host-side, out of scope)")

    convert = getattr(dataset, "convert_targets", None)
    lut_np = lut_from_convert_targets(convert) if convert is not None else None
    lut = torch.from_numpy(lut_np).to(device) if lut_np is not None else None
    mean = getattr(dataset, "mean", CITYSCAPES_MEAN)
    std = getattr(dataset, "std", CITYSCAPES_STD)
    rank, world = world_info(process_group)
    lo, hi = shard_bounds(len(dataset.img_ids), rank, world)

    def load_raw(push_iter):
        img_id = dataset.img_ids[push_iter]
        with open(dataset.get_img_path(img_id), "rb") as f:
            img = Image.open(f).convert("RGB")
        margin = dataset.image_margin_size
        img = img.crop((margin, margin, img.width - margin, img.height - margin))
        gt_ann = np.load(os.path.join(dataset.annotations_dir, img_id + ".npy"))
        if convert is not None and lut is None:
            gt_ann = convert(gt_ann)
        labels = torch.as_tensor(np.ascontiguousarray(gt_ann)).to(device)
        if labels.dtype not in (torch.int64, torch.int32, torch.uint8):
            labels = labels.to(torch.int64)
        return to_normalized_tensor(img, mean, std).unsqueeze(0).to(device), labels

    def load(push_iter):
        img_tensor, labels = load_raw(push_iter)
        return ppnet.conv_features(img_tensor), labels

    scan_runs = {}  # image index -> the image indices of the backbone batch the scan ran it in

    def load_as_scanned(push_iter):
        """The image's features as the scan computed them: its whole scan batch through the
        backbone again (a batch-of-1 convolution need not equal the batched one bit for bit,
        and the exact-tie resolution compares distances exactly)."""
        ids = scan_runs.get(push_iter, [push_iter])
        raw = [load_raw(i) for i in ids]
        feats = scan_features(ppnet.conv_features(torch.cat([r[0] for r in raw], 0)))
        k = ids.index(push_iter)
        return feats[k:k + 1], raw[k][1]

    log("Updating prototypes...")
    per = max(1, int(images_per_batch))
    with torch.no_grad():
        # Runs of up to images_per_batch consecutive images of one geometry go through the
        # backbone as one batch and through mask -> argmin -> merge as ONE push_update call;
        # the merge folds them in image order, so the result is the serial scan's.
        run: List[tuple] = []

        def flush():
            if run:
                imgs = torch.cat([r[0] for r in run], 0)
                labels = torch.stack([r[1] for r in run], 0)
                push_update(state, scan_features(ppnet.conv_features(imgs)), labels, ppnet.prototype_vectors, proto_class_t,
                            run[0][2], lut, words)
                ids = [r[2] for r in run]
                for i in ids:
                    scan_runs[i] = ids
                run.clear()

        for push_iter in range(lo, hi):
            img_tensor, labels = load_raw(push_iter)
            if run and (len(run) == per or run[0][0].shape != img_tensor.shape or run[0][1].shape != labels.shape
                        or run[0][1].dtype != labels.dtype):
                flush()
            run.append((img_tensor, labels, push_iter))
        flush()

    # exact ties inside a winning image, in the reference's set order (this rank's winners,
    # before the shards merge: the owner's patch travels with its key)
    with torch.no_grad():
        moved = resolve_exact_ties(state, load_as_scanned, ppnet.prototype_vectors, proto_class_t, lut, log=log)
    if moved:
        log(f"\t{len(moved)} exact tie(s) resolved in the reference's patch order: {moved[:20]}")
    if world > 1:
        reduce_push_state(state, process_group)
    state.near_ties = near_ties(state, ppnet.prototype_vectors)
    if len(state.near_ties):
        log(f"\t{len(state.near_ties)} prototype(s) won by a margin within f32 rounding of the runner-up patch: "
            f"{state.near_ties.tolist()[:20]}")

    with_class = bool(save_prototype_class_identity)
    proto_rf_boxes = rf_boxes(state, proto_class, with_class)
    # push.py:309-343: bound boxes on each prototype's winning image (this rank's shard only).
    proto_bound_boxes = np.full_like(proto_rf_boxes, -1)
    winners = proto_rf_boxes[:, 0]
    mine = np.unique(winners[(winners >= lo) & (winners < hi)])
    with torch.no_grad():
        def items():
            for img_idx in mine:
                conv_features, labels = load(int(img_idx))
                yield np.nonzero(winners == img_idx)[0], conv_features, labels
        boxes = batch_bound_boxes(items(), ppnet.prototype_vectors, proto_class, proto_rf_boxes,
                                  ppnet.prototype_activation_function, ppnet.epsilon,
                                  prototype_activation_function_in_numpy, lut)
    for j, b in boxes.items():
        proto_bound_boxes[j, 0] = winners[j]
        proto_bound_boxes[j, 1:5] = b
        if with_class:
            proto_bound_boxes[j, 5] = proto_class[j]
    if world > 1:
        proto_bound_boxes = reduce_bound_boxes(proto_bound_boxes, device, process_group)
    if proto_epoch_dir is not None and proto_bound_boxes_filename_prefix is not None:
        np.save(os.path.join(proto_epoch_dir, f"{proto_bound_boxes_filename_prefix}-receptive_field{epoch_number}.npy"),
                proto_rf_boxes)
        np.save(os.path.join(proto_epoch_dir, f"{proto_bound_boxes_filename_prefix}{epoch_number}.npy"),
                proto_bound_boxes)

    log("\tExecuting push ...")
    dedup_and_prune(ppnet, state.fmap.cpu().numpy(), root_dir_for_saving_prototypes, log)
    log(f"\tpush time: \t{time.time() - start}")
    return state
