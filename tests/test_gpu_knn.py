"""Parity of the HIP k-nearest-patch search and pruning (find_nearest.py:66-342, prune.py:11-109)
with the oracle. Bar: bit-exact — the label resize (PIL NEAREST), the f64 masked minima and their
first-index argmin, the patch labels, the heap contents and order (heapq's tie behaviour
included) and the prune list — for the same distance maps."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import knn_oracle as kn
from oracle import push_oracle as pu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

pytestmark = pytest.mark.gpu


def _knn():
    from protoseg_amd import knn
    return knn


def _lut():
    lut = np.full(34, 0, dtype=np.int32)
    for k, v in pu.CITYSCAPES_19_EVAL_CATEGORIES.items():
        lut[k] = v
    return lut


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32, torch.uint8])
@pytest.mark.parametrize("H,W,h,w", [(1024, 2048, 129, 257), (513, 513, 65, 65), (60, 110, 9, 13), (5, 7, 20, 30)])
def test_resize_label_matches_pil(device, dtype, H, W, h, w):
    knn = _knn()
    rng = np.random.default_rng(H + w)
    lab = rng.integers(0, 20, size=(2, H, W))
    out = knn.resize_label(torch.from_numpy(lab).to(dtype).to(device), h, w).cpu().numpy()
    for i in range(2):
        assert np.array_equal(out[i], kn.resize_label(lab[i], h, w))


def test_resize_label_lut(device):
    knn = _knn()
    raw = np.random.default_rng(1).integers(0, 34, size=(1, 100, 200))
    lut = _lut()
    out = knn.resize_label(torch.from_numpy(raw).to(device), 13, 25, torch.from_numpy(lut).to(device)).cpu().numpy()
    assert np.array_equal(out[0], kn.resize_label(lut[raw[0]], 13, 25))


def test_image_min_exact(device):
    """f64 masked minimum and first argmin equal numpy's, including an all-void image, -0.0 and
    exact ties inside one map (quantised distances)."""
    knn = _knn()
    dists, labels = kn.synthetic_search(4, 37, 33, 65, 33, 65, 6, seed=3, ties=True)
    labels[1][:] = 0
    dists[2][5] = -0.0
    d = torch.from_numpy(np.stack(dists)).to(device)
    small = torch.from_numpy(np.stack(labels)).to(torch.int32).to(device)  # map size == label size
    m, i = knn.image_min(d, small)
    m, i = m.cpu().numpy(), i.cpu().numpy()
    for b in range(4):
        em, ei = kn.image_min(dists[b], labels[b] - 1)
        assert np.array_equal(m[b], em) and np.array_equal(i[b], ei)
    assert np.all(m[1] >= 1e7)


@pytest.mark.parametrize("H,W,h,w", [(60, 110, 9, 13), (1024, 2048, 129, 257), (7, 9, 20, 30)])
def test_patch_labels_exact(device, H, W, h, w):
    """Boxes of non-integer size (1024 / 129), empty boxes (map larger than the image) and the
    vote rules, against the oracle for every (image, prototype)."""
    knn = _knn()
    P, K = 23, 5
    rng = np.random.default_rng(h)
    _, labels = kn.synthetic_search(3, 1, 1, 1, H, W, K, seed=h)
    idx = rng.integers(0, h * w, size=(3, P)).astype(np.int32)
    pc = (np.arange(P) % K).astype(np.int32)
    out = knn.patch_labels(torch.from_numpy(idx).to(device), h, w, torch.from_numpy(np.stack(labels)).to(device),
                           torch.from_numpy(pc).to(device)).cpu().numpy()
    for b in range(3):
        sy = labels[b] - 1
        for j in range(P):
            exp = kn.patch_label(sy, kn.patch_box(int(idx[b, j]), H, W, h, w), int(pc[j]))
            assert out[b, j] == (knn.SKIP if exp is None else exp), (b, j)


def _run_gpu(knn, device, dists, labels, proto_class, k, batch, lut=None, threshold=0):
    P = len(proto_class)
    pc = torch.from_numpy(proto_class).to(device)
    state = knn.KnnState.create(P, k, device)
    lut_t = torch.from_numpy(lut).to(device) if lut is not None else None
    for b0 in range(0, len(dists), batch):
        d = torch.from_numpy(np.stack(dists[b0:b0 + batch])).to(device)
        y = torch.from_numpy(np.stack(labels[b0:b0 + batch])).to(device)
        knn.knn_update(state, d, y, pc, b0, lut_t)
    res = knn.knn_finalize(state, pc, threshold)
    return {kk: v.cpu().numpy() for kk, v in res.items()}


def test_knn_matches_golden(device):
    knn = _knn()
    g = np.load(os.path.join(GOLDEN, "knn_small.npz"))
    res = _run_gpu(knn, device, list(g["dist"]), list(g["labels"]), g["proto_class"], int(g["k"]), 1,
                   threshold=int(g["prune_threshold"]))
    for key in ("dist", "label", "img", "patch"):
        assert np.array_equal(res[key], g["out_" + key]), key
    assert list(np.nonzero(res["prune"])[0]) == list(g["pruned"])


@pytest.mark.parametrize("k,batch,ties", [(1, 3, False), (5, 4, True), (12, 1, True), (64, 7, False)])
def test_knn_multi_batch_vs_oracle(device, k, batch, ties):
    """Heaps carried across batches of different sizes; quantised distances force equal minima
    across images (heapq's eviction order decides)."""
    knn = _knn()
    n, P, K = 15, 41, 6
    dists, labels = kn.synthetic_search(n, P, 11, 17, 70, 120, K, seed=k + batch, ties=ties)
    labels[3][:] = 0
    dists[9] = dists[4].copy()
    proto_class = (np.arange(P) % K).astype(np.int32)
    exp = kn.find_k_nearest(dists, [y - 1 for y in labels], proto_class, k)
    res = _run_gpu(knn, device, dists, labels, proto_class, k, batch, threshold=2)
    for key in ("dist", "label", "img", "patch"):
        e = exp[key]
        if key == "label":
            e = np.where(exp["img"] < 0, knn.SKIP, e)
        assert np.array_equal(res[key], e), key
    assert list(np.nonzero(res["prune"])[0]) == kn.prune_list(exp["label"], proto_class, 2)


def test_knn_raw_ids_through_lut(device):
    """Raw Cityscapes ids with the CLS_CONVERT table == labels converted on the host."""
    knn = _knn()
    lut = _lut()
    rng = np.random.default_rng(2)
    dists, _ = kn.synthetic_search(5, 19, 9, 13, 1, 1, 19, seed=2)
    raw = [rng.integers(0, 34, size=(60, 110)) for _ in range(5)]
    proto_class = np.arange(19, dtype=np.int32)
    a = _run_gpu(knn, device, dists, raw, proto_class, 3, 2, lut=lut)
    b = _run_gpu(knn, device, dists, [lut[r] for r in raw], proto_class, 3, 2)
    for key in a:
        assert np.array_equal(a[key], b[key]), key
    exp = kn.find_k_nearest(dists, [lut[r] - 1 for r in raw], proto_class, 3)
    assert np.array_equal(a["img"], exp["img"]) and np.array_equal(a["label"], exp["label"])


def test_knn_on_layer_distances(device):
    """The product pipeline: distances from the HIP l2 kernel (push_forward), then the search; the
    oracle runs on the same device-computed maps."""
    from protoseg_amd import ops
    knn = _knn()
    gen = torch.Generator().manual_seed(0)
    n, C, h, w, P, K = 6, 64, 33, 65, 38, 19
    x = torch.rand(n, C, h, w, generator=gen).to(device)
    protos = torch.rand(P, C, 1, 1, generator=gen).to(device)
    dist = ops.l2_distances(x, protos)
    _, labels = kn.synthetic_search(n, 1, 1, 1, 260, 520, K, seed=9)
    proto_class = (np.arange(P) // 2).astype(np.int32)
    d_np = list(dist.float().cpu().numpy())
    res = _run_gpu(knn, device, d_np, labels, proto_class, 4, 3)
    exp = kn.find_k_nearest(d_np, [y - 1 for y in labels], proto_class, 4)
    for key in ("dist", "label", "img", "patch"):
        assert np.array_equal(res[key], exp[key]), key


def test_prune_prototypes_drop_in(device, tmp_path):
    """prune.py:11-109 end to end on a tiny on-disk dataset: the k-NN labels, prune_info.npy,
    prototypes_to_keep.json and the pruned model agree with the oracle on the model's own maps."""
    from PIL import Image

    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    from protoseg_amd.knn import prune_prototypes
    from protoseg_amd.model import PPNet

    torch.manual_seed(0)
    feats = deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[])
    net = PPNet(feats, 513, (38, 64, 1, 1), None, 19, add_on_layers_type="deeplab_simple").to(device)
    rng = np.random.default_rng(4)
    img_dir, ann_dir = tmp_path / "img", tmp_path / "ann"
    img_dir.mkdir()
    ann_dir.mkdir()

    class DS:
        img_ids = [f"im{i}" for i in range(4)]
        image_margin_size = 4
        annotations_dir = str(ann_dir)

        def get_img_path(self, img_id):
            return str(img_dir / f"{img_id}.png")

    ds = DS()
    for i, img_id in enumerate(ds.img_ids):
        Image.fromarray(rng.integers(0, 256, size=(72, 104, 3), dtype=np.uint8)).save(ds.get_img_path(img_id))
        np.save(ann_dir / f"{img_id}.npy", rng.integers(0, 20, size=(64, 96)).astype(np.int64))
    net.eval()
    from protoseg_amd.push import to_normalized_tensor
    maps, ys = [], []
    with torch.no_grad():
        for img_id in ds.img_ids:
            img = Image.open(ds.get_img_path(img_id)).convert("RGB").crop((4, 4, 100, 68))
            maps.append(net.push_forward(to_normalized_tensor(img).unsqueeze(0).to(device))[1][0].cpu().numpy())
            ys.append(np.load(ann_dir / f"{img_id}.npy") - 1)
    pc = net.prototype_class_identity.argmax(1).numpy().astype(np.int32)
    exp = kn.find_k_nearest(maps, ys, pc, 3)
    pruned = kn.prune_list(exp["label"], pc, 1)

    info = prune_prototypes(ds, net, 3, 1, None, str(tmp_path / "model"), 7, log=lambda *_: None)
    assert np.array_equal(np.load(tmp_path / "model" / "img" / "full_class_id.npy"), exp["label"])
    assert list(info[:, 0]) == pruned and list(info[:, 1]) == [int(pc[j]) for j in pruned]
    keep = json.load(open(tmp_path / "model" / "prototypes_to_keep.json"))
    assert keep == [j for j in range(38) if j not in pruned]
    assert net.num_prototypes == 38 - len(pruned)
    saved = np.load(tmp_path / "model" / "pruned_prototypes_epoch7_k3_pt1" / "prune_info.npy")
    assert np.array_equal(saved, info)
