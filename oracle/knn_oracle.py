"""ORACLE — test infrastructure only. CPU restatement of the k-nearest-patch search and pruning.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline; the product path never calls it.

Restates, per image in dataset order:
  find_nearest.py:113-116   search_y = convert_targets(y) - 1 (void -> -1)
  find_nearest.py:128-132   interpolated_y = resize_label(search_y, (w, h)) (PIL NEAREST,
                            segmentation/dataset.py:23-31); proto_dist_ + 10e6 * (y == -1) (f64)
  find_nearest.py:136-145   per prototype j: np.amin / np.argmin of its masked map
  find_nearest.py:159-180   patch box int(r * H/h) .. int((r+1) * H/h); empty box -> skip
  find_nearest.py:202-211   label = class of j if any box pixel has it, else the most common value
  find_nearest.py:224-230   heapq.heappush while < k, else heappushpop (ImagePatch.__lt__ on
                            negative distance, find_nearest.py:44-61)
  find_nearest.py:227-232   heaps[j].sort(); heaps[j][::-1]
  prune.py:35-43            prune j if Counter(labels_j)[class_j] < prune_threshold
  model.py:311-336          prune_prototypes keeps sorted(set(range(P)) - set(pruned))
This runs the very heapq / list.sort / numpy calls the reference makes (Python's own heapq and
PIL are the same libraries the reference calls), so the oracle is the reference's algorithm on
the same inputs. Parity status: UNPINNED against the reference itself (its Python may not be
imported here; it ships no tests or fixtures for this path); PIL's NEAREST index
sequence is pinned against PIL in tests/test_knn_oracle.py.
"""
from __future__ import annotations

import heapq
from collections import Counter
from typing import Dict, List, Optional, Sequence

import numpy as np


def resize_label(label: np.ndarray, h: int, w: int) -> np.ndarray:
    """segmentation/dataset.py:30-31: PIL NEAREST resize of the label map to (w, h)."""
    from PIL import Image
    return np.asarray(Image.fromarray(label.astype(float)).resize((w, h), resample=Image.NEAREST)).astype(np.int64)


def pil_nearest_index(n_in: int, n_out: int) -> np.ndarray:
    """PIL's NEAREST source indices (ImagingScaleAffine): start at scale / 2, add scale in f64
    per output step, truncate. The HIP resize kernel replays exactly this sequence."""
    a = n_in / n_out
    xo = a * 0.5
    out = np.empty(n_out, np.int64)
    for x in range(n_out):
        out[x] = int(xo)
        xo += a
    return np.minimum(out, n_in - 1)


class ImagePatch:
    """find_nearest.py:44-61: ordered by negative distance only."""

    def __init__(self, label, distance, img, patch):
        self.label = label
        self.negative_distance = -distance
        self.img = img
        self.patch = patch

    def __lt__(self, other):
        return self.negative_distance < other.negative_distance


def image_min(dist: np.ndarray, small_y: Optional[np.ndarray]) -> (np.ndarray, np.ndarray):
    """dist [P, h, w] f32, small_y [h, w] (search_y resized, void -1) -> per prototype
    (np.amin, np.argmin) of the masked map (find_nearest.py:132, 140, 143-145)."""
    d = dist if small_y is None else dist + 10e6 * (small_y == -1)[None]
    flat = d.reshape(d.shape[0], -1)
    return np.amin(flat, axis=1), np.argmin(flat, axis=1)


def patch_box(idx: int, H: int, W: int, h: int, w: int):
    """find_nearest.py:119-120, 143-166: the pixel box of flat patch idx (clamped like slicing)."""
    r, c = np.unravel_index(idx, (h, w))
    ph, pw = H / h, W / w
    return (int(r * ph), min(int((r + 1) * ph), H), int(c * pw), min(int((c + 1) * pw), W))


def patch_label(search_y: np.ndarray, box, target_class: int):
    """find_nearest.py:202-211 (None for an empty box, find_nearest.py:179-180)."""
    r0, r1, c0, c1 = box
    labels = search_y[r0:r1, c0:c1]
    if labels.size == 0:
        return None
    if np.any(labels == target_class):
        return target_class
    values, counts = np.unique(labels, return_counts=True)
    return int(values[np.argmax(counts)])


def find_k_nearest(dists: Sequence[np.ndarray], search_ys: Sequence[np.ndarray], proto_class: np.ndarray, k: int,
                   small_ys: Optional[Sequence[np.ndarray]] = None) -> Dict[str, np.ndarray]:
    """dists: per image [P, h, w] f32 distance maps; search_ys: per image [H, W] converted labels
    MINUS ONE (void -1); proto_class [P]. small_ys: per image [h, w] resized search_y (default:
    resize_label of search_y, as the reference). Returns [P, k] arrays in the reference's final
    order (ascending distance): dist (f64), label, img, patch (flat map index); slots past a
    heap's size: inf / None-marker INT32_MIN / -1 / -1."""
    P = len(proto_class)
    heaps: List[list] = [[] for _ in range(P)]
    for img, (dist, sy) in enumerate(zip(dists, search_ys)):
        h, w = dist.shape[1:]
        H, W = sy.shape
        small = resize_label(sy, h, w) if small_ys is None else small_ys[img]
        dmin, idx = image_min(dist, small)
        for j in range(P):
            box = patch_box(int(idx[j]), H, W, h, w)
            label = patch_label(sy, box, int(proto_class[j]))
            if label is None:
                continue
            item = ImagePatch(label, dmin[j], img, int(idx[j]))
            if len(heaps[j]) < k:
                heapq.heappush(heaps[j], item)
            else:
                heapq.heappushpop(heaps[j], item)
    out = {"dist": np.full((P, k), np.inf), "label": np.full((P, k), np.iinfo(np.int32).min, np.int64),
           "img": np.full((P, k), -1, np.int64), "patch": np.full((P, k), -1, np.int64)}
    for j in range(P):
        heaps[j].sort()
        heaps[j] = heaps[j][::-1]
        for q, it in enumerate(heaps[j]):
            out["dist"][j, q] = -it.negative_distance
            out["label"][j, q] = it.label
            out["img"][j, q] = it.img
            out["patch"][j, q] = it.patch
    return out


def prune_list(labels: np.ndarray, proto_class: np.ndarray, prune_threshold: int) -> List[int]:
    """prune.py:35-43 on the [P, k] nearest-patch labels."""
    pruned = []
    for j in range(len(proto_class)):
        if Counter(labels[j].tolist())[int(proto_class[j])] < prune_threshold:
            pruned.append(j)
    return pruned


def synthetic_search(n_img: int, P: int, h: int, w: int, H: int, W: int, K: int, seed: int, void_frac=0.3,
                     ties: bool = False):
    """Seeded distance maps and blocky label maps (converted labels, 0 = void); with ties the
    distances are quantised so that equal minima occur across images and patches."""
    rng = np.random.default_rng(seed)
    dists, labels = [], []
    for _ in range(n_img):
        d = rng.random((P, h, w), dtype=np.float32) * 50
        if ties:
            d = np.floor(d / 10).astype(np.float32)
        dists.append(d)
        bh, bw = max(1, H // 6), max(1, W // 6)
        blocks = rng.integers(1, K + 1, size=((H + bh - 1) // bh, (W + bw - 1) // bw))
        blocks[rng.random(blocks.shape) < void_frac] = 0
        labels.append(np.repeat(np.repeat(blocks, bh, 0), bw, 1)[:H, :W].astype(np.int64))
    return dists, labels
