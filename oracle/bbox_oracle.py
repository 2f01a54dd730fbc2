"""ORACLE — test infrastructure only. CPU restatement of the push high-activation bound boxes.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.

Restates segmentation/push.py:309-343 and helpers.py:48-82:
  * ``activation_map``: push.py:312-316 verbatim numpy (np.log((d + 1) / (d + eps)) on the f32
    map, or max_dist - d);
  * ``cv2_resize_cubic``: cv2.resize(act, (W, H), interpolation=cv2.INTER_CUBIC), push.py:318.
    cv2 is NOT installed here and the reference cannot be run, so this follows
    OpenCV's published resize.cpp algorithm: fx = (float)((dx + 0.5) * scale - 0.5) with
    scale = 1 / (dsize / ssize) in f64, sx = floor(fx), interpolateCubic(fx - sx) with
    A = -0.75 in f32, taps sx-1..sx+2 clamped to the border, a horizontal pass then a vertical
    pass, each a left-to-right f32 sum of separately rounded products. Parity with cv2 itself
    is UNPINNED (its SIMD paths may fuse or reorder); the kernel is held to this restatement;
  * ``np.percentile(upsampled, 95)`` is called as the reference calls it (push.py:322);
  * ``find_continuous_high_activation_crop``: helpers.py:48-82 loop for loop.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np

F = np.float32


def activation_map(dist: np.ndarray, kind: str = "log", eps: float = 1e-4, max_dist: float = 64) -> np.ndarray:
    """push.py:312-316 (``dist`` f32 [h, w])."""
    d = np.asarray(dist, dtype=np.float32)
    if kind == "log":
        return np.log((d + 1) / (d + eps))
    if kind == "linear":
        return max_dist - d
    raise ValueError(kind)


def _cubic_coeffs(x: np.ndarray) -> np.ndarray:
    """OpenCV interpolateCubic, A = -0.75, f32, each operation rounded."""
    A = F(-0.75)
    x = x.astype(np.float32)
    x1 = x + F(1)
    c0 = ((A * x1 - F(5) * A) * x1 + F(8) * A) * x1 - F(4) * A
    c1 = ((A + F(2)) * x - (A + F(3))) * x * x + F(1)
    omx = F(1) - x
    c2 = ((A + F(2)) * omx - (A + F(3))) * omx * omx + F(1)
    c3 = F(1) - c0 - c1 - c2
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.float32)


def _taps(n_dst: int, n_src: int) -> Tuple[np.ndarray, np.ndarray]:
    scale = 1.0 / (float(n_dst) / float(n_src))
    f = ((np.arange(n_dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    fl = np.floor(f)
    coeffs = _cubic_coeffs((f - fl).astype(np.float32))
    idx = fl.astype(np.int64)[:, None] + np.arange(-1, 3)[None, :]
    return np.clip(idx, 0, n_src - 1), coeffs


def cv2_resize_cubic(src: np.ndarray, H: int, W: int) -> np.ndarray:
    """cv2.resize(src, dsize=(W, H), interpolation=cv2.INTER_CUBIC) for a 2-D f32 map."""
    S = np.asarray(src, dtype=np.float32)
    xi, a = _taps(W, S.shape[1])
    yi, b = _taps(H, S.shape[0])
    # horizontal pass over every source row: ((S0*a0 + S1*a1) + S2*a2) + S3*a3
    hr = S[:, xi[:, 0]] * a[:, 0]
    for k in range(1, 4):
        hr = hr + S[:, xi[:, k]] * a[:, k]
    # vertical pass
    out = hr[yi[:, 0], :] * b[:, 0:1]
    for k in range(1, 4):
        out = out + hr[yi[:, k], :] * b[:, k:k + 1]
    return out.astype(np.float32)


def find_continuous_high_activation_crop(activation_map, patch_bbox: Sequence[int], threshold, add_margin=5):
    """helpers.py:48-82."""
    start_h, end_h, start_w, end_w = tuple(int(v) for v in patch_bbox)
    mask = (activation_map >= threshold).astype(int)
    stopped = [False, False, False, False]
    while not all(stopped):
        if not stopped[0] and start_h > 0 and np.amax(mask[start_h - 1, start_w:end_w + 1]) > 0.5:
            start_h = start_h - 1
        else:
            stopped[0] = True
        if not stopped[1] and end_h < activation_map.shape[0] - 1 and np.amax(mask[end_h + 1, start_w:end_w + 1]) > 0.5:
            end_h = end_h + 1
        else:
            stopped[1] = True
        if not stopped[2] and start_w > 0 and np.amax(mask[start_h:end_h + 1, start_w - 1]) > 0.5:
            start_w = start_w - 1
        else:
            stopped[2] = True
        if not stopped[3] and end_w < activation_map.shape[1] - 1 and np.amax(mask[start_h:end_h + 1, end_w + 1]) > 0.5:
            end_w = end_w + 1
        else:
            stopped[3] = True
    start_h = max(start_h - add_margin, 0)
    start_w = max(start_w - add_margin, 0)
    end_h = min(end_h + add_margin, activation_map.shape[0] - 1)
    end_w = min(end_w + add_margin, activation_map.shape[1] - 1)
    return start_h, end_h + 1, start_w, end_w + 1


def bound_box_from_upsampled(upsampled: np.ndarray, img_y: np.ndarray, target_class: int,
                             rf: Sequence[int], percentile: float = 95) -> Tuple[np.float32, Tuple[int, ...]]:
    """push.py:321-329 given the upsampled activation map: (threshold, proto_bound_j)."""
    threshold = np.percentile(upsampled, percentile)
    y_mask = np.asarray(img_y) == (target_class + 1)
    gt = upsampled * y_mask
    return threshold, find_continuous_high_activation_crop(gt, rf, threshold=threshold)


def bound_box(dist: np.ndarray, img_y: np.ndarray, target_class: int, rf: Sequence[int], kind: str = "log",
              eps: float = 1e-4, max_dist: float = 64):
    """push.py:309-329 end to end for one prototype: (threshold, box, upsampled)."""
    act = activation_map(dist, kind, eps, max_dist)
    up = cv2_resize_cubic(act, img_y.shape[0], img_y.shape[1])
    thr, box = bound_box_from_upsampled(up, img_y, target_class, rf)
    return thr, box, up


def rf_box(patch_i: int, patch_j: int, H: int, W: int, h: int, w: int) -> Tuple[int, int, int, int]:
    """push.py:288-292 (float64 patch arithmetic)."""
    ph, pw = H / h, W / w
    return (int(patch_i * ph), int(patch_i * ph + ph) + 1, int(patch_j * pw), int(patch_j * pw + pw) + 1)
