"""Parity of the bound-box kernels (bbox.hip) with the oracle (push.py:309-343, helpers.py:48-82).

Bar: the activation map within 2 ulp of numpy's f32 np.log (the kernel rounds an f64 log; numpy
uses its own f32 log); the cubic upsample of the kernel's activations bit-exact with the
restatement; thresholds bit-exact with np.percentile of the kernel's upsampled map; boxes exact.
End-to-end (distances -> boxes) the boxes equal the oracle's on these seeds.
"""
import numpy as np
import pytest
import torch

from oracle import bbox_oracle as bo

pytestmark = pytest.mark.gpu


def _push():
    from protoseg_amd import push
    return push


def _maps(rng, m, h, w):
    d = (rng.random((m, h, w)) * 4).astype(np.float32)
    d[:, h // 2, w // 3] = 0.0
    return d


def _labels(rng, H, W, n=1):
    y = rng.integers(0, 20, size=(n, H, W)).astype(np.int64)
    y[:, H // 4: 3 * H // 4, W // 5: 4 * W // 5] = 4  # one big region of class index 3
    return y


@pytest.mark.parametrize("kind", ["log", "linear"])
@pytest.mark.parametrize("h,w,H,W", [(9, 17, 64, 128), (7, 11, 57, 93), (65, 65, 513, 513), (33, 70, 300, 1100),
                                     (40, 30, 20, 12)])
def test_act_upsample_vs_oracle(device, kind, h, w, H, W):
    push = _push()
    rng = np.random.default_rng(h * W)
    d = _maps(rng, 3, h, w)
    act, up = push.act_upsample(torch.from_numpy(d).to(device), H, W, kind, 1e-4, 64.0)
    act, up = act.cpu().numpy(), up.cpu().numpy()
    for j in range(3):
        ref = bo.activation_map(d[j], kind, 1e-4, 64)
        assert np.allclose(act[j], ref, rtol=2.5e-7, atol=0), np.abs(act[j] - ref).max()
        assert np.array_equal(up[j], bo.cv2_resize_cubic(act[j], H, W))


@pytest.mark.parametrize("ldtype", [torch.int64, torch.int32, torch.uint8])
@pytest.mark.parametrize("q", [95.0, 50.0, 100.0, 0.0])
def test_bound_boxes_vs_oracle(device, ldtype, q):
    push = _push()
    rng = np.random.default_rng(int(q) + 7)
    h, w, H, W = 9, 17, 72, 136
    m = 6
    d = _maps(rng, m, h, w)
    y = _labels(rng, H, W, n=2)
    li = np.array([0, 1, 1, 0, 1, 0], np.int32)
    tc = np.array([3, 3, 0, 5, 18, 3], np.int32)
    rf = np.array([bo.rf_box(r, c, H, W, h, w) for r, c in [(4, 5), (0, 0), (8, 16), (3, 9), (6, 2), (8, 0)]],
                  np.int32)
    _, up = push.act_upsample(torch.from_numpy(d).to(device), H, W)
    thr, box = push.bound_boxes(up, torch.from_numpy(y).to(ldtype).to(device), torch.from_numpy(tc).to(device),
                                torch.from_numpy(rf).to(device), torch.from_numpy(li).to(device), percentile=q)
    up, thr, box = up.cpu().numpy(), thr.cpu().numpy(), box.cpu().numpy()
    for j in range(m):
        t = np.percentile(up[j], q)
        assert thr[j] == t, (j, thr[j], t)
        mask = up[j] * (y[li[j]] == tc[j] + 1)
        assert tuple(box[j]) == bo.find_continuous_high_activation_crop(mask, rf[j], t), j


@pytest.mark.parametrize("H,W", [(63, 129), (1, 5), (33, 1)])
def test_bound_boxes_ragged_and_ties(device, H, W):
    push = _push()
    rng = np.random.default_rng(H + W)
    up = np.round(rng.random((3, H, W)) * 4).astype(np.float32) / 4  # few distinct values: ties
    up[1] = 1.0  # constant map
    y = rng.integers(0, 3, size=(H, W)).astype(np.int64)
    tc = np.array([0, 1, 0], np.int32)
    rf = np.array([[0, 1, 0, 1], [H // 2, H // 2 + 1, W // 2, W // 2 + 1], [H - 1, H, W - 1, W]], np.int32)
    thr, box = push.bound_boxes(torch.from_numpy(up).to(device), torch.from_numpy(y).to(device),
                                torch.from_numpy(tc).to(device), torch.from_numpy(rf).to(device), margin=2)
    thr, box = thr.cpu().numpy(), box.cpu().numpy()
    for j in range(3):
        t = np.percentile(up[j], 95)
        assert thr[j] == t
        exp = bo.find_continuous_high_activation_crop(up[j] * (y == tc[j] + 1), rf[j], t, add_margin=2)
        assert tuple(box[j]) == exp


def test_bound_boxes_lut_and_invalid_rows(device):
    push = _push()
    from oracle import push_oracle as pu
    rng = np.random.default_rng(11)
    H, W = 40, 64
    raw = rng.integers(0, 29, size=(H, W)).astype(np.uint8)
    raw[10:30, 20:50] = 7  # raw id 7 -> eval class 5
    conv = pu.convert_targets(raw)
    lut = np.full(29, -1, np.int32)
    for k, v in pu.CITYSCAPES_19_EVAL_CATEGORIES.items():
        lut[k] = v
    up = rng.random((3, H, W)).astype(np.float32)
    tc = np.array([4, 4, 4], np.int32)
    rf = np.array([[15, 16, 30, 31], [-1, 2, 0, 1], [0, 1, W, W + 1]], np.int32)
    li = np.array([0, 0, 0], np.int32)
    thr, box = push.bound_boxes(torch.from_numpy(up).to(device), torch.from_numpy(raw).to(device),
                                torch.from_numpy(tc).to(device), torch.from_numpy(rf).to(device),
                                torch.from_numpy(li).to(device), lut=torch.from_numpy(lut).to(device))
    thr, box = thr.cpu().numpy(), box.cpu().numpy()
    t = np.percentile(up[0], 95)
    assert thr[0] == t
    assert tuple(box[0]) == bo.find_continuous_high_activation_crop(up[0] * (conv == 5), rf[0], t)
    assert (box[1:] == -1).all() and np.isnan(thr[1:]).all()


def test_bound_boxes_full_resolution_end_to_end(device):
    """1024x2048 image, 129x257 map (push.py:275): distances -> boxes against the oracle chain."""
    push = _push()
    rng = np.random.default_rng(2975)
    h, w, H, W = 129, 257, 1024, 2048
    d = (rng.random((3, h, w)) * 6 + 0.5).astype(np.float32)
    cells = [(60, 100), (5, 250), (128, 0)]
    for j, (r, c) in enumerate(cells):
        d[j, max(r - 3, 0):r + 4, max(c - 6, 0):c + 7] *= 0.05  # a blob of near patches
        d[j, r, c] = 0.0
    y = np.zeros((1, H, W), np.uint8)
    y[0, 300:700, 500:1500] = 8
    y[0, :64, 1900:] = 8
    y[0, 960:, :200] = 8
    tc = np.full(3, 7, np.int32)
    rf = np.array([bo.rf_box(r, c, H, W, h, w) for r, c in cells], np.int32)
    _, up = push.act_upsample(torch.from_numpy(d).to(device), H, W)
    thr, box = push.bound_boxes(up, torch.from_numpy(y).to(device), torch.from_numpy(tc).to(device),
                                torch.from_numpy(rf).to(device))
    up, thr, box = up.cpu().numpy(), thr.cpu().numpy(), box.cpu().numpy()
    for j in range(3):
        t_ref, box_ref, up_ref = bo.bound_box(d[j], y[0], 7, rf[j])
        assert np.allclose(up[j], up_ref, rtol=1e-6, atol=1e-6)
        assert thr[j] == np.percentile(up[j], 95)
        assert abs(float(thr[j]) - float(t_ref)) <= 1e-6 * abs(float(t_ref))
        assert tuple(box[j]) == box_ref, (j, box[j], box_ref)


def test_batch_bound_boxes_more_winners_than_one_f32_call(device):
    """P = 570 (30 prototypes/class): 450 prototypes win on one image, more than one f32 layer
    call holds (384 at C = 64); the sliced distance calls give the boxes of per-slice calls."""
    push = _push()
    rng = np.random.default_rng(570)
    C, h, w, H, W, P = 64, 9, 17, 72, 136, 570
    x = torch.from_numpy(rng.random((1, C, h, w)).astype(np.float32)).to(device)
    protos = torch.from_numpy(rng.random((P, C)).astype(np.float32)).to(device)
    y = torch.from_numpy(_labels(rng, H, W)[0]).to(device)
    pc = np.arange(P) // 30
    ids = np.arange(450) * 570 // 450
    rfb = np.zeros((P, 6), np.int64)
    rfb[:, 1:5] = [bo.rf_box(int(j) % h, int(j) % w, H, W, h, w) for j in range(P)]
    whole = push.batch_bound_boxes([(ids, x, y)], protos, pc, rfb)
    parts = {}
    for s in range(0, len(ids), 150):
        parts.update(push.batch_bound_boxes([(ids[s:s + 150], x, y)], protos, pc, rfb))
    assert len(whole) == len(ids) and whole == parts


def test_push_prototypes_writes_bound_boxes(device, tmp_path):
    """push_prototypes end to end: proto_bound_boxes (push.py:338-343) from each prototype's
    winning image equal the oracle chain on that image's distances."""
    from PIL import Image

    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    from protoseg_amd.model import PPNet
    from protoseg_amd.push import push_prototypes, to_normalized_tensor

    torch.manual_seed(0)
    feats = deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[])
    net = PPNet(feats, 513, (38, 64, 1, 1), None, 19, add_on_layers_type="deeplab_simple").to(device)
    rng = np.random.default_rng(9)
    img_dir, ann_dir = tmp_path / "img", tmp_path / "ann"
    img_dir.mkdir()
    ann_dir.mkdir()

    class DS:
        img_ids = [f"im{i}" for i in range(3)]
        image_margin_size = 4
        annotations_dir = str(ann_dir)

        def get_img_path(self, img_id):
            return str(img_dir / f"{img_id}.png")

    ds = DS()
    for img_id in ds.img_ids:
        Image.fromarray(rng.integers(0, 256, size=(72, 104, 3), dtype=np.uint8)).save(ds.get_img_path(img_id))
        np.save(ann_dir / f"{img_id}.npy", rng.integers(0, 20, size=(64, 96)).astype(np.int64))
    net.eval()
    with torch.no_grad():
        dists = []
        for img_id in ds.img_ids:
            img = Image.open(ds.get_img_path(img_id)).convert("RGB").crop((4, 4, 100, 68))
            x = net.conv_features(to_normalized_tensor(img).unsqueeze(0).to(device))
            from protoseg_amd.ops import l2_distances
            dists.append(l2_distances(x, net.prototype_vectors, net.epsilon, precision="f32")[0].cpu().numpy())
    out = tmp_path / "protos"
    push_prototypes(ds, net, root_dir_for_saving_prototypes=str(out), epoch_number=3,
                    proto_bound_boxes_filename_prefix="bb", log=lambda *_: None)
    rf = np.load(out / "epoch-3" / "bb-receptive_field3.npy")
    bb = np.load(out / "epoch-3" / "bb3.npy")
    assert bb.shape == rf.shape == (38, 6)
    pc = bb[:, 5]
    checked = 0
    for j in range(38):
        if rf[j, 0] < 0:
            assert (bb[j] == -1).all()
            continue
        img = int(rf[j, 0])
        y = np.load(ann_dir / f"{ds.img_ids[img]}.npy")
        _, box, _ = bo.bound_box(dists[img][j], y, int(pc[j]), rf[j, 1:5])
        assert bb[j, 0] == img and bb[j, 5] == rf[j, 5]
        assert tuple(bb[j, 1:5]) == box, (j, bb[j], box)
        checked += 1
    assert checked > 10


def test_bound_boxes_match_committed_golden(device):
    """tests/golden/bbox_small.npz: the kernels' upsampled maps within 1e-6 of the golden ones
    (the log differs from numpy's by <= 1 ulp), thresholds / boxes equal to the golden values."""
    import os
    push = _push()
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bbox_small.npz"))
    H, W = g["labels"].shape
    _, up = push.act_upsample(torch.from_numpy(g["dist"]).to(device), H, W, "log", 1e-4, 64.0)
    thr, box = push.bound_boxes(up, torch.from_numpy(g["labels"]).to(device),
                                torch.from_numpy(g["proto_class"]).to(device),
                                torch.from_numpy(g["rf"].astype(np.int32)).to(device))
    up, thr, box = up.cpu().numpy(), thr.cpu().numpy(), box.cpu().numpy()
    assert np.allclose(up, g["up"], rtol=1e-6, atol=1e-6)
    assert np.allclose(thr, g["threshold"], rtol=1e-6, atol=0)
    assert np.array_equal(box, g["box"])
