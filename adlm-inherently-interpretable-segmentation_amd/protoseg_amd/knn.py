"""k-nearest-patch search and prototype pruning on the HIP kernels.

Drop-ins for find_nearest.py:66-342 (``find_k_nearest_patches_to_prototypes``) and
prune.py:11-109 (``prune_prototypes``). The reference copies every image's [P, h, w] distance
map to the host and loops over prototypes in Python (np.amin / np.argmin, a label vote over the
patch box, heapq); here each batch is four launches and the heaps stay on the device:
  resize_label      PIL NEAREST label resize (segmentation/dataset.py:23-31)
  knn_image_min     masked f64 min / first argmin per (image, prototype)
  knn_patch_label   patch box + label vote per (image, prototype)
  knn_heap_push     heapq.heappush / heappushpop per prototype, CPython's sift order
and ``knn_finalize`` sorts the heaps (find_nearest.py:227-232) and applies the pruning rule
(prune.py:35-43). Results equal the reference's for the same distance maps, ties included.

Out of scope (host-side visualisation, needs cv2/matplotlib): the PNG outputs of
find_nearest.py:240-322; with ``full_save`` the numeric outputs are written (act patterns,
class_id.npy, full_class_id.npy).
"""
from __future__ import annotations

import json
import os
import shutil
import time
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np
import torch
from torch import Tensor

from . import _lib

SKIP = -(2 ** 31)  # patch_label of an image whose patch box is empty (never offered to a heap)


def _label_dtype(t: Tensor) -> int:
    return {torch.int64: _lib.I64, torch.int32: _lib.I32, torch.uint8: _lib.U8}.get(t.dtype, -1)


def _labels3(labels: Tensor) -> Tensor:
    if labels.dim() == 2:
        labels = labels.unsqueeze(0)
    if _label_dtype(labels) < 0:
        labels = labels.to(torch.int64)
    return labels.contiguous()


def resize_label(labels: Tensor, h: int, w: int, lut: Optional[Tensor] = None) -> Tensor:
    """segmentation/dataset.py:23-31 on the device: labels [n, H, W] (or [H, W]) -> int32
    [n, h, w] by PIL NEAREST (bit-exact index sequence), mapped through ``lut`` when given."""
    dev = _lib.require_device(labels, lut)
    labels = _labels3(labels)
    n, H, W = labels.shape
    out = torch.empty((n, h, w), device=dev, dtype=torch.int32)
    lut_c = lut.to(torch.int32).contiguous() if lut is not None else None
    with torch.cuda.device(dev):
        _lib.call("protoseg_resize_label", _lib.ptr(labels), _label_dtype(labels), n, H, W, h, w, _lib.ptr(lut_c),
                  0 if lut_c is None else lut_c.numel(), _lib.ptr(out), _lib.stream_of(dev))
    return out


@dataclass
class KnnState:
    """Per-prototype heaps of the k nearest images (find_nearest.py:84-88), device-resident."""
    k: int
    neg: Tensor     # [P, k] f64 negative distances (ImagePatch.negative_distance)
    label: Tensor   # [P, k] int32 patch labels
    patch: Tensor   # [P, k] int32 flat map index of the closest patch
    img: Tensor     # [P, k] int64 dataset index
    size: Tensor    # [P] int32
    status: Tensor  # [1] int32, bit 0: a label outside [-256, 255]

    @classmethod
    def create(cls, P: int, k: int, device) -> "KnnState":
        if not 1 <= k <= 64:
            raise _lib.ProtosegError(f"k={k} outside [1, 64]")
        z = dict(device=device)
        return cls(k=k, neg=torch.zeros((P, k), dtype=torch.float64, **z),
                   label=torch.zeros((P, k), dtype=torch.int32, **z), patch=torch.zeros((P, k), dtype=torch.int32, **z),
                   img=torch.zeros((P, k), dtype=torch.int64, **z), size=torch.zeros(P, dtype=torch.int32, **z),
                   status=torch.zeros(1, dtype=torch.int32, **z))


def image_min(distances: Tensor, small_labels: Optional[Tensor]):
    """find_nearest.py:132, 140-145: (min f64 [n, P], argmin int32 [n, P]) of the distance maps
    [n, P, h, w] with 10e6 added on void patches (small_labels [n, h, w] int32, 0 = void)."""
    dev = _lib.require_device(distances, small_labels)
    d = distances.float().contiguous()
    n, P, h, w = d.shape
    sl = small_labels.to(torch.int32).contiguous() if small_labels is not None else None
    min_dist = torch.empty((n, P), device=dev, dtype=torch.float64)
    min_idx = torch.empty((n, P), device=dev, dtype=torch.int32)
    with torch.cuda.device(dev):
        _lib.call("protoseg_knn_image_min", _lib.ptr(d), n, P, h, w, _lib.ptr(sl), _lib.ptr(min_dist),
                  _lib.ptr(min_idx), _lib.stream_of(dev))
    return min_dist, min_idx


def patch_labels(min_idx: Tensor, h: int, w: int, labels: Tensor, proto_class: Tensor,
                 lut: Optional[Tensor] = None, status: Optional[Tensor] = None) -> Tensor:
    """find_nearest.py:159-166, 202-211: label of each winning patch [n, P] int32 (SKIP for an
    empty box). labels [n, H, W] full-resolution (converted, or raw with ``lut``)."""
    dev = _lib.require_device(min_idx, labels, proto_class, lut, status)
    labels = _labels3(labels)
    n, H, W = labels.shape
    P = min_idx.shape[1]
    out = torch.empty((n, P), device=dev, dtype=torch.int32)
    st = status if status is not None else torch.zeros(1, device=dev, dtype=torch.int32)
    lut_c = lut.to(torch.int32).contiguous() if lut is not None else None
    with torch.cuda.device(dev):
        _lib.call("protoseg_knn_patch_label", _lib.ptr(min_idx.contiguous()), n, P, h, w, _lib.ptr(labels),
                  _label_dtype(labels), H, W, _lib.ptr(lut_c), 0 if lut_c is None else lut_c.numel(),
                  _lib.ptr(proto_class.to(torch.int32).contiguous()), _lib.ptr(out), _lib.ptr(st),
                  _lib.stream_of(dev))
    return out


def knn_update(state: KnnState, distances: Tensor, labels: Tensor, proto_class: Tensor, first_img: int,
               lut: Optional[Tensor] = None) -> None:
    """One batch of images (dataset indices first_img ..): distances [n, P, h, w] (push_forward),
    labels [n, H, W]. Resize -> masked min -> patch label -> heap push, all on the device."""
    labels = _labels3(labels)
    n, P, h, w = distances.shape
    small = resize_label(labels, h, w, lut)
    min_dist, min_idx = image_min(distances, small)
    plab = patch_labels(min_idx, h, w, labels, proto_class, lut, state.status)
    dev = distances.device
    with torch.cuda.device(dev):
        _lib.call("protoseg_knn_heap_push", _lib.ptr(min_dist), _lib.ptr(min_idx), _lib.ptr(plab), n, int(first_img),
                  P, state.k, _lib.ptr(state.neg), _lib.ptr(state.label), _lib.ptr(state.patch), _lib.ptr(state.img),
                  _lib.ptr(state.size), _lib.stream_of(dev))


def knn_finalize(state: KnnState, proto_class: Tensor, prune_threshold: int = 0):
    """find_nearest.py:227-232 + prune.py:35-43 -> dict of [P, k] device tensors (dist f64,
    label, img, patch; ascending distance) plus class_count [P] and prune [P] (bool)."""
    dev = _lib.require_device(state.neg, proto_class)
    P, k = state.neg.shape
    out = dict(dist=torch.empty((P, k), device=dev, dtype=torch.float64),
               label=torch.empty((P, k), device=dev, dtype=torch.int32),
               img=torch.empty((P, k), device=dev, dtype=torch.int64),
               patch=torch.empty((P, k), device=dev, dtype=torch.int32),
               class_count=torch.empty(P, device=dev, dtype=torch.int32),
               prune=torch.empty(P, device=dev, dtype=torch.int32))
    with torch.cuda.device(dev):
        _lib.call("protoseg_knn_finalize", _lib.ptr(state.neg), _lib.ptr(state.label), _lib.ptr(state.patch),
                  _lib.ptr(state.img), _lib.ptr(state.size), P, k, _lib.ptr(proto_class.to(torch.int32).contiguous()),
                  int(prune_threshold), _lib.ptr(out["dist"]), _lib.ptr(out["label"]), _lib.ptr(out["img"]),
                  _lib.ptr(out["patch"]), _lib.ptr(out["class_count"]), _lib.ptr(out["prune"]), _lib.stream_of(dev))
    if int(state.status.item()) & 1:
        raise _lib.ProtosegError("a label outside [-256, 255] (after convert_targets - 1) was seen")
    out["prune"] = out["prune"].bool()
    return out


def _prototype_classes(ppnet) -> Tensor:
    return torch.argmax(ppnet.prototype_class_identity, dim=1).to(torch.int32)


def find_k_nearest_patches_to_prototypes(dataset, prototype_network_parallel, k=5, preprocess_input_function=None,
                                         full_save=False, root_dir_for_saving_images="./nearest", log=print,
                                         prototype_activation_function_in_numpy=None, prune_threshold=0):
    """Drop-in for find_nearest.py:66-342: returns labels_all_prototype [P, k] (numpy int). With
    ``full_save`` writes the numeric outputs (per prototype ``nearest-i_act.npy`` and
    ``class_id.npy``, then ``full_class_id.npy``); the PNGs are not produced. The activation
    pattern is recomputed for the k winners only, from their stored image indices."""
    from PIL import Image

    from .push import CITYSCAPES_MEAN, CITYSCAPES_STD, lut_from_convert_targets, to_normalized_tensor

    ppnet = prototype_network_parallel.module if hasattr(prototype_network_parallel, "module") \
        else prototype_network_parallel
    ppnet.eval()
    log("find nearest patches")
    start = time.time()
    device = ppnet.prototype_vectors.device
    P = ppnet.num_prototypes
    proto_class = _prototype_classes(ppnet).to(device)
    state = KnnState.create(P, k, device)
    convert = getattr(dataset, "convert_targets", None)
    lut_np = lut_from_convert_targets(convert) if convert is not None else None
    lut = torch.from_numpy(lut_np).to(device) if lut_np is not None else None
    mean = getattr(dataset, "mean", CITYSCAPES_MEAN)
    std = getattr(dataset, "std", CITYSCAPES_STD)

    def load(i):
        img_id = dataset.img_ids[i]
        with open(dataset.get_img_path(img_id), "rb") as f:
            img = Image.open(f).convert("RGB")
        m = dataset.image_margin_size
        img = img.crop((m, m, img.width - m, img.height - m))
        y = np.load(os.path.join(dataset.annotations_dir, img_id + ".npy"))
        if convert is not None and lut is None:
            y = convert(np.expand_dims(y, 0))[0]
        labels = torch.as_tensor(np.ascontiguousarray(y)).to(device)
        return img, labels

    with torch.no_grad():
        for i in range(len(dataset.img_ids)):
            img, labels = load(i)
            x = to_normalized_tensor(img, mean, std).unsqueeze(0).to(device)
            _, dist = ppnet.push_forward(x)
            knn_update(state, dist, labels, proto_class, i, lut)
    res = knn_finalize(state, proto_class, prune_threshold)
    labels_all = res["label"].cpu().numpy().astype(np.int64)

    if full_save:
        os.makedirs(root_dir_for_saving_images, exist_ok=True)
        imgs = res["img"].cpu().numpy()
        eps = float(getattr(ppnet, "epsilon", 1e-4))
        act_fn = getattr(ppnet, "prototype_activation_function", "log")
        max_dist = int(np.prod(ppnet.prototype_shape[1:]))
        cache = {}
        with torch.no_grad():
            for j in range(P):
                d_j = os.path.join(root_dir_for_saving_images, str(j))
                os.makedirs(d_j, exist_ok=True)
                for q in range(k):
                    i = int(imgs[j, q])
                    if i < 0:
                        continue
                    if i not in cache:
                        img, _ = load(i)
                        x = to_normalized_tensor(img, mean, std).unsqueeze(0).to(device)
                        cache = {i: ppnet.push_forward(x)[1][0].double().cpu().numpy()}
                    dm = cache[i][j]
                    if act_fn == "log":                                   # find_nearest.py:187-189
                        act = np.log((dm + 1) / (dm + eps))
                    elif act_fn == "linear":
                        act = max_dist - dm
                    else:
                        act = prototype_activation_function_in_numpy(dm)
                    np.save(os.path.join(d_j, f"nearest-{q + 1}_act.npy"), act)
                np.save(os.path.join(d_j, "class_id.npy"), labels_all[j])
        np.save(os.path.join(root_dir_for_saving_images, "full_class_id.npy"), labels_all)

    log(f"\tfind nearest patches time: \t{time.time() - start}")
    find_k_nearest_patches_to_prototypes.last_result = res
    return labels_all


def prune_prototypes(dataset, prototype_network_parallel, k, prune_threshold, preprocess_input_function,
                     original_model_dir, epoch_number, log: Callable = print, copy_prototype_imgs=True):
    """Drop-in for prune.py:11-109: k-NN search (full_save), prune prototypes whose k nearest
    patches hold fewer than ``prune_threshold`` of their class, bookkeeping files, model prune."""
    ppnet = prototype_network_parallel.module if hasattr(prototype_network_parallel, "module") \
        else prototype_network_parallel
    find_k_nearest_patches_to_prototypes(dataset, prototype_network_parallel, k=k,
                                         preprocess_input_function=preprocess_input_function, full_save=True,
                                         root_dir_for_saving_images=os.path.join(original_model_dir, "img"), log=log,
                                         prune_threshold=prune_threshold)
    res = find_k_nearest_patches_to_prototypes.last_result
    original_num_prototypes = ppnet.num_prototypes
    prune_flags = res["prune"].cpu().numpy()
    prototypes_to_prune: List[int] = [int(j) for j in np.nonzero(prune_flags)[0]]
    log(f"k = {k}, prune_threshold = {prune_threshold}")
    log(f"{len(prototypes_to_prune)} prototypes will be pruned")

    classes = _prototype_classes(ppnet).cpu().numpy()
    prune_info = np.hstack((np.array(prototypes_to_prune, dtype=np.int64).reshape(-1, 1),
                            classes[prototypes_to_prune].astype(np.int64).reshape(-1, 1)))
    sub = os.path.join(original_model_dir, f"pruned_prototypes_epoch{epoch_number}_k{k}_pt{prune_threshold}")
    os.makedirs(sub, exist_ok=True)
    np.save(os.path.join(sub, "prune_info.npy"), prune_info)

    ppnet.prune_prototypes(prototypes_to_prune)
    prototypes_to_keep = sorted(set(range(original_num_prototypes)) - set(prototypes_to_prune))
    log(f"Prototypes to keep: {prototypes_to_keep}")
    with open(os.path.join(original_model_dir, "prototypes_to_keep.json"), "w") as fp:
        json.dump(prototypes_to_keep, fp)

    if copy_prototype_imgs:  # prune.py:78-107, for whichever of the files exist
        src_dir = os.path.join(original_model_dir, "img", f"epoch-{epoch_number}")
        dst_dir = os.path.join(sub, "img", f"epoch-{epoch_number}")
        os.makedirs(dst_dir, exist_ok=True)
        for idx, j in enumerate(prototypes_to_keep):
            for pat in ("prototype-img%d.png", "prototype-img-original%d.png",
                        "prototype-img-original_with_self_act%d.png", "prototype-self-act%d.npy"):
                src = os.path.join(src_dir, pat % j)
                if os.path.exists(src):
                    shutil.copyfile(src, os.path.join(dst_dir, pat % idx))
        for name in (f"bb{epoch_number}.npy", f"bb-receptive_field{epoch_number}.npy"):
            src = os.path.join(src_dir, name)
            if os.path.exists(src):
                np.save(os.path.join(dst_dir, name), np.load(src)[prototypes_to_keep])
    return prune_info
