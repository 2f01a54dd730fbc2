"""CPU: pin the k-NN / pruning oracle (find_nearest.py:66-342, prune.py:11-109 restated) — PIL's
NEAREST index sequence, an independent sort-based restatement for distinct distances, the
reference's tie and skip rules, the committed golden vector — and the C ABI's validation."""
import ctypes
import os

import numpy as np
import pytest

from oracle import knn_oracle as kn

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("n_in,n_out", [(1024, 129), (2048, 257), (513, 65), (65, 513), (7, 7), (100, 3),
                                        (3, 100), (1, 5), (997, 131)])
def test_pil_nearest_index_matches_pil(n_in, n_out):
    """The index sequence the HIP resize kernel replays equals PIL's own resize (both axes)."""
    lab = np.arange(n_in, dtype=np.int64)
    cols = kn.resize_label(lab[None, :].repeat(2, 0), 2, n_out)[0]
    rows = kn.resize_label(lab[:, None].repeat(2, 1), n_out, 2)[:, 0]
    idx = kn.pil_nearest_index(n_in, n_out)
    assert np.array_equal(cols, idx) and np.array_equal(rows, idx)


def test_pil_nearest_random_shapes():
    rng = np.random.default_rng(5)
    for _ in range(60):
        H, W, h, w = (int(v) for v in rng.integers(1, 300, 4))
        lab = rng.integers(-1, 20, size=(H, W))
        exp = lab[kn.pil_nearest_index(H, h)][:, kn.pil_nearest_index(W, w)]
        assert np.array_equal(kn.resize_label(lab, h, w), exp)


def _sorted_restatement(dists, search_ys, proto_class, k):
    """Independent restatement for distinct distances: per prototype, the k smallest image minima
    in ascending order (what the heap + sort + reverse computes when nothing ties)."""
    P = len(proto_class)
    cand = [[] for _ in range(P)]
    for img, (d, sy) in enumerate(zip(dists, search_ys)):
        h, w = d.shape[1:]
        small = kn.resize_label(sy, h, w)
        masked = d.astype(np.float64) + 1e7 * (small == -1)[None]
        for j in range(P):
            flat = masked[j].ravel()
            i = int(np.argmin(flat))
            box = kn.patch_box(i, sy.shape[0], sy.shape[1], h, w)
            lab = kn.patch_label(sy, box, int(proto_class[j]))
            if lab is not None:
                cand[j].append((float(flat[i]), img, i, lab))
    out = []
    for j in range(P):
        out.append(sorted(cand[j])[:k])
    return out


@pytest.mark.parametrize("k", [1, 3, 8])
def test_oracle_matches_sorted_restatement(k):
    dists, labels = kn.synthetic_search(6, 11, 7, 9, 40, 50, 5, seed=k)
    labels[2][:] = 0  # all void
    proto_class = (np.arange(11) * 5 // 11).astype(np.int32)
    res = kn.find_k_nearest(dists, [y - 1 for y in labels], proto_class, k)
    ref = _sorted_restatement(dists, [y - 1 for y in labels], proto_class, k)
    for j in range(11):
        n = len(ref[j])
        assert np.array_equal(res["dist"][j, :n], [r[0] for r in ref[j]])
        assert np.array_equal(res["img"][j, :n], [r[1] for r in ref[j]])
        assert np.array_equal(res["patch"][j, :n], [r[2] for r in ref[j]])
        assert np.array_equal(res["label"][j, :n], [r[3] for r in ref[j]])
        assert np.all(res["img"][j, n:] == -1)


def test_void_mask_and_label_vote_rules():
    """find_nearest.py:132: a void patch loses to any labelled one; an all-void image still
    yields its (masked) minimum. 202-211: own class wins the vote; else the most common value,
    the smaller on a tie."""
    d = np.array([[[0.5, 3.0], [2.0, 9.0]]], np.float32)       # P=1, 2x2 map
    y = np.array([[-1, 4], [4, 4]])                              # search_y, map size == image size
    m, i = kn.image_min(d, y)
    assert m[0] == 2.0 and i[0] == 2
    m, i = kn.image_min(d, np.full((2, 2), -1))
    assert m[0] == np.float64(np.float32(0.5)) + 1e7 and i[0] == 0
    sy = np.array([[1, 1, 2, 2, -1, -1]])
    assert kn.patch_label(sy, (0, 1, 0, 6), 2) == 2
    assert kn.patch_label(sy, (0, 1, 0, 6), 7) == -1             # three-way tie -> smallest value
    assert kn.patch_label(sy, (0, 1, 0, 4), 7) == 1
    assert kn.patch_label(sy, (0, 1, 3, 3), 7) is None           # empty box -> skipped


def test_heap_ties_follow_heapq():
    """heappushpop replaces the root only on a strictly smaller distance (image 2 is rejected), and
    the root it evicts is whichever equal item the heap holds there (image 0, not image 1); the
    final stable sort + reverse lists the later of two kept equals first."""
    P, h, w, H, W = 1, 2, 2, 4, 4
    d = [np.full((P, h, w), v, np.float32) for v in (1.0, 1.0, 1.0, 0.5)]
    y = [np.zeros((H, W), np.int64) for _ in d]
    res = kn.find_k_nearest(d, y, np.zeros(1, np.int32), 2)
    assert list(res["img"][0]) == [3, 1]
    res = kn.find_k_nearest(d[:3], y[:3], np.zeros(1, np.int32), 2)
    assert list(res["img"][0]) == [1, 0]


def test_prune_rule():
    labels = np.array([[0, 0, 1], [1, 1, 1], [2, -1, 2]])
    assert kn.prune_list(labels, np.array([0, 0, 2]), 2) == [1]
    assert kn.prune_list(labels, np.array([0, 0, 2]), 3) == [0, 1, 2]


def test_oracle_reproduces_golden():
    g = np.load(os.path.join(GOLDEN, "knn_small.npz"))
    res = kn.find_k_nearest(list(g["dist"]), [y - 1 for y in g["labels"]], g["proto_class"], int(g["k"]))
    for key in ("dist", "label", "img", "patch"):
        assert np.array_equal(res[key], g["out_" + key]), key
    assert kn.prune_list(res["label"], g["proto_class"], int(g["prune_threshold"])) == list(g["pruned"])


def test_knn_abi_validation_without_gpu():
    from protoseg_amd import _lib
    lib = _lib.load()
    null, dummy = ctypes.c_void_p(None), ctypes.c_void_p(256)
    assert lib.protoseg_resize_label(null, _lib.I64, 1, 8, 8, 4, 4, null, 0, dummy, null) == _lib.ERR_INVALID
    assert lib.protoseg_resize_label(dummy, _lib.F32, 1, 8, 8, 4, 4, null, 0, dummy, null) == _lib.ERR_UNSUPPORTED
    assert lib.protoseg_knn_image_min(dummy, 0, 4, 2, 2, null, dummy, dummy, null) == _lib.ERR_INVALID
    st = lib.protoseg_knn_heap_push(dummy, dummy, dummy, 1, 0, 4, 65, dummy, dummy, dummy, dummy, dummy, null)
    assert st == _lib.ERR_UNSUPPORTED and b"k=65" in lib.protoseg_last_error()
    st = lib.protoseg_knn_patch_label(dummy, 1, 4, 2, 2, dummy, _lib.I64, 8, 8, null, 0, null, dummy, dummy, null)
    assert st == _lib.ERR_INVALID
    st = lib.protoseg_knn_finalize(dummy, dummy, dummy, dummy, dummy, 4, 0, dummy, 1, dummy, dummy, dummy, dummy,
                                   dummy, dummy, null)
    assert st == _lib.ERR_UNSUPPORTED
