"""CPU checks of the bound-box oracle (segmentation/push.py:309-343, helpers.py:48-82).

cv2 is absent, so the INTER_CUBIC restatement is cross-checked against torch's bicubic
interpolate (align_corners=False), which implements the same kernel (A = -0.75, half-pixel
centres, clamped border taps); the two differ only in f32 rounding order (tolerance 1e-5
relative to the map's range). The greedy crop is pinned by hand-worked known answers.
"""
import numpy as np
import pytest
import torch

from oracle import bbox_oracle as bo


@pytest.mark.parametrize("h,w,H,W", [(9, 17, 64, 128), (5, 7, 37, 61), (17, 17, 136, 136), (33, 65, 256, 512)])
def test_cubic_restatement_matches_torch_bicubic(h, w, H, W):
    src = np.random.default_rng(h * w).standard_normal((h, w)).astype(np.float32)
    ours = bo.cv2_resize_cubic(src, H, W)
    ref = torch.nn.functional.interpolate(torch.from_numpy(src)[None, None].double(), size=(H, W), mode="bicubic",
                                          align_corners=False)[0, 0].numpy()
    assert ours.dtype == np.float32 and ours.shape == (H, W)
    assert np.abs(ours - ref).max() <= 1e-5 * (np.abs(src).max() + 1)


def test_cubic_restatement_constant_and_identity():
    c = np.full((6, 9), 2.5, np.float32)
    assert np.allclose(bo.cv2_resize_cubic(c, 48, 72), 2.5, atol=1e-6)
    src = np.random.default_rng(1).random((7, 5)).astype(np.float32)
    assert np.array_equal(bo.cv2_resize_cubic(src, 7, 5), src)  # same size: taps (0, 1, 0, 0)


def _percentile_f32(a, q):
    """What bound_box_kernel computes: numpy 'linear' percentile in f32 arithmetic."""
    a = np.sort(a.ravel())
    n = a.size
    v = np.float32(n - 1) * (np.float32(q) / np.float32(100))
    if v >= np.float32(n - 1):
        lo = hi = n - 1
    else:
        lo = int(np.floor(v))
        hi = lo + 1
    g = np.float32(v - np.floor(v))
    A, B = a[lo], a[hi]
    d = np.float32(B - A)
    return np.float32(B - d * (np.float32(1) - g)) if g >= 0.5 else np.float32(A + d * g)


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 4225, 33153, 2097152])
@pytest.mark.parametrize("q", [95.0, 0.0, 50.0, 100.0, 99.9])
def test_percentile_f32_rule_is_numpys(n, q):
    rng = np.random.default_rng(n)
    a = (rng.random(n) * 9).astype(np.float32)
    if n > 10:
        a[: n // 3] = a[0]  # ties
    got = _percentile_f32(a, q)
    ref = np.percentile(a, q)
    assert ref.dtype == np.float32 and got == ref


def test_crop_known_answers():
    m = np.zeros((20, 30), np.float32)
    m[5:10, 10:15] = 1.0
    assert bo.find_continuous_high_activation_crop(m, (7, 8, 12, 13), 0.5, add_margin=0) == (5, 10, 10, 15)
    assert bo.find_continuous_high_activation_crop(m, (7, 8, 12, 13), 0.5) == (0, 15, 5, 20)
    # an isolated hot pixel outside the touching region does not pull the box
    m[0, 0] = 1.0
    assert bo.find_continuous_high_activation_crop(m, (7, 8, 12, 13), 0.5, add_margin=0) == (5, 10, 10, 15)
    # rf box reaching past the map (end index = H, as push.py:289 can produce) stops at once
    z = np.zeros((20, 30), np.float32)
    assert bo.find_continuous_high_activation_crop(z, (18, 20, 27, 30), 0.5) == (13, 20, 22, 30)
    # threshold <= 0: masked-out pixels (0) count, the box grows to the whole map
    assert bo.find_continuous_high_activation_crop(z, (3, 4, 3, 4), 0.0, add_margin=0) == (0, 20, 0, 30)


def test_bound_box_end_to_end_prototype_on_its_patch():
    rng = np.random.default_rng(5)
    h, w, H, W = 9, 17, 72, 136
    dist = rng.random((h, w)).astype(np.float32) * 5 + 1
    dist[4, 8] = 0.0  # the winning patch
    y = np.zeros((H, W), np.int64)
    y[20:50, 40:100] = 3
    rf = bo.rf_box(4, 8, H, W, h, w)
    thr, box, up = bo.bound_box(dist, y, 2, rf)
    assert up.shape == (H, W) and thr == np.percentile(up, 95)
    assert box[0] <= rf[0] and box[1] >= min(rf[1], H - 1) and box[2] <= rf[2] and box[3] >= min(rf[3], W - 1)


def test_oracle_reproduces_committed_golden():
    """tests/golden/bbox_small.npz (make_golden.py) is re-derived bit for bit."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bbox_small.npz"))
    for j in range(g["dist"].shape[0]):
        t, b, u = bo.bound_box(g["dist"][j], g["labels"], int(g["proto_class"][j]), g["rf"][j], "log", 1e-4, 64)
        assert np.array_equal(u, g["up"][j]) and t == g["threshold"][j] and tuple(b) == tuple(g["box"][j])
