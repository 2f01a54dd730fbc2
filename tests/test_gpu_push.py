"""Parity of the HIP push kernels with the push oracle (segmentation/push.py restated).

Bar: bit-exact for the integer work (patch class masks, winning patch / image indices, rf
boxes, dedup). Winning distances and feature vectors are compared exactly where the oracle's
minimum is separated from the runner-up by more than the f32 rounding bound of the distance;
inside that bound either candidate is a correct answer of the same computation and the test
checks that the kernel's pick is one of them.
"""
import os

import numpy as np
import pytest
import torch

from oracle import protoseg_oracle as po
from oracle import push_oracle as pu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

pytestmark = pytest.mark.gpu


def _push():
    from protoseg_amd import push
    return push


def _lut():
    lut = np.full(29, -1, dtype=np.int32)
    for k, v in pu.CITYSCAPES_19_EVAL_CATEGORIES.items():
        lut[k] = v
    return torch.from_numpy(lut)


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32, torch.uint8])
def test_patch_mask_matches_golden(device, dtype):
    push = _push()
    g = np.load(os.path.join(GOLDEN, "push_small.npz"))
    labels = torch.from_numpy(g["labels"]).to(dtype).to(device)
    mask = push.patch_class_mask(labels, 8, 16)
    assert np.array_equal(mask.cpu().numpy().view(np.uint32), g["mask"])
    raw = torch.from_numpy(g["raw_labels"]).to(dtype).to(device)
    mask_lut = push.patch_class_mask(raw, 8, 16, _lut().to(device))
    assert np.array_equal(mask_lut.cpu().numpy().view(np.uint32), g["mask"])


@pytest.mark.parametrize("H,W,h,w", [(1024, 2048, 129, 257), (513, 513, 65, 65), (100, 37, 13, 5), (7, 9, 7, 9)])
def test_patch_mask_vs_oracle_geometry(device, H, W, h, w):
    """Non-integer patch sizes (1024/129 = 7.94): the float64 pixel->patch division must match."""
    push = _push()
    rng = np.random.default_rng(H + W)
    labels = rng.integers(0, 20, size=(2, H, W)).astype(np.int64)
    labels[:, : H // 3] = 0  # a void band
    mask = push.patch_class_mask(torch.from_numpy(labels).to(device), h, w).cpu().numpy().view(np.uint32)
    for i in range(2):
        assert np.array_equal(mask[i], pu.class_patch_bitmask_fast(labels[i], h, w))
    if H * W <= 100 * 37:
        sets = pu.class_to_patch_index_dict(labels[0], h, w, 19)
        assert np.array_equal(mask[0], pu.bitmask_from_dict(sets, h, w))


def test_push_matches_golden_serial_scan(device):
    """3 images scanned in order: winners, distances, feature vectors and rf boxes."""
    push = _push()
    g = np.load(os.path.join(GOLDEN, "push_small.npz"))
    x = torch.from_numpy(g["x"]).to(device)
    protos = torch.from_numpy(g["protos"]).to(device)
    pc = torch.from_numpy(g["proto_class"]).to(device)
    labels = torch.from_numpy(g["labels"]).to(device)
    P, C = protos.shape
    state = push.PushState.create(P, C, device)
    for i in range(x.shape[0]):  # one image per call, as push_prototypes does
        push.push_update(state, x[i:i + 1], labels[i], protos, pc, i)
    _check_against_oracle(state, g, push)
    # the same scan as one batched call
    state_b = push.PushState.create(P, C, device)
    push.push_update(state_b, x, labels, protos, pc, 0)
    for a, b in ((state.dist, state_b.dist), (state.img, state_b.img), (state.patch, state_b.patch),
                 (state.fmap, state_b.fmap)):
        assert torch.equal(a, b)


def _check_against_oracle(state, g, push):
    ref_d = g["global_min_proto_dist"]
    dist = state.dist.cpu().numpy().astype(np.float64)
    img = state.img.cpu().numpy()
    patch = state.patch.cpu().numpy()
    boxes = push.rf_boxes(state, g["proto_class"])
    ref_boxes = g["proto_rf_boxes"]
    n_img, _, h, w = g["x"].shape
    for j in range(ref_d.shape[0]):
        if np.isinf(ref_d[j]):
            assert img[j] == -1 and np.isinf(dist[j])
            continue
        # the reference's own candidates for prototype j and their runner-up gap
        cand = []
        for i in range(n_img):
            member = (g["mask"][i] >> g["proto_class"][j]) & 1
            d = g["dist"][i, j].reshape(-1)
            cand += [(d[q], i, q) for q in np.nonzero(member)[0]]
        cand.sort()
        bound = 1e-5 * (1.0 + abs(cand[0][0])) + 4e-6 * 64
        if len(cand) == 1 or cand[1][0] - cand[0][0] > bound:
            assert (img[j], patch[j]) == (ref_boxes[j, 0], g["winner_patch"][j]), f"prototype {j}"
            assert np.array_equal(boxes[j], ref_boxes[j])
            assert np.array_equal(state.fmap[j].cpu().numpy(), g["global_min_fmap_patches"][j].astype(np.float32))
        else:
            near = {(i, q) for d, i, q in cand if d - cand[0][0] <= bound}
            assert (img[j], patch[j]) in near
        assert abs(dist[j] - ref_d[j]) <= bound


def test_push_multi_image_vs_oracle_loop(device):
    """Random 2-image scan against the literal Python loop of push.py (small images)."""
    push = _push()
    n_img, C, H, W, h, w, P, K = 2, 64, 40, 72, 10, 18, 57, 19
    gen = torch.Generator().manual_seed(31)
    x = torch.sigmoid(2 * torch.randn(n_img, C, h, w, generator=gen))
    protos = torch.rand(P, C, generator=gen)
    pc = torch.argmax(po.class_identity(P, K), dim=1).numpy().astype(np.int32)
    labels = np.random.default_rng(3).integers(0, K + 1, size=(n_img, H, W)).astype(np.int64)
    ost = pu.PushOracleState(P, C)
    dists, masks = [], []
    for i in range(n_img):
        d = po.l2_convolution(x[i:i + 1], protos[:, :, None, None], torch.ones(P, C, 1, 1))[0]
        sets = pu.class_to_patch_index_dict(labels[i], h, w, K)
        pu.update_prototypes_on_image_core(ost, x[i].numpy(), d.permute(1, 2, 0).numpy(), labels[i], pc, K, i, sets)
        dists.append(d.numpy())
        masks.append(pu.bitmask_from_dict(sets, h, w))
    g = dict(x=x.numpy(), proto_class=pc, dist=np.stack(dists), mask=np.stack(masks),
             global_min_proto_dist=ost.global_min_proto_dist,
             global_min_fmap_patches=ost.global_min_fmap_patches.reshape(P, C), winner_patch=ost.winner_patch,
             proto_rf_boxes=ost.proto_rf_boxes)
    state = push.PushState.create(P, C, device)
    push.push_update(state, x.to(device), torch.from_numpy(labels).to(device), protos.to(device),
                     torch.from_numpy(pc).to(device), 0)
    _check_against_oracle(state, g, push)


@pytest.mark.parametrize("n_img", [1, 8])
def test_push_full_resolution_properties(device, n_img):
    """1024x2048 labels, 129x257 maps, 190 prototypes, one image per call and an 8-image batch:
    each key is the masked minimum of the float64 brute-force distances and lies in the
    prototype's class mask; wherever that minimum is separated from its runner-up by more than
    the f32 rounding bound of the expanded distance, the patch index is exactly the argmin
    (push.py:255-263: np.argmin over the masked class distances)."""
    push = _push()
    C, H, W, h, w, P, K = 64, 1024, 2048, 129, 257, 190, 19
    gen = torch.Generator().manual_seed(37 + n_img)
    x = torch.sigmoid(2 * torch.randn(n_img, C, h, w, generator=gen))
    protos = torch.rand(P, C, generator=gen)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32)
    rng = np.random.default_rng(41 + n_img)
    labels = np.repeat(np.repeat(rng.integers(0, K + 1, size=(n_img, H // 16, W // 16)), 16, 1), 16, 2).astype(np.uint8)
    mask = push.patch_class_mask(torch.from_numpy(labels).to(device), h, w)
    keys = push.push_argmin(x.to(device), protos.to(device), pc.to(device), mask)
    mm = mask.cpu().numpy().view(np.uint32)
    exact_idx = 0
    for i in range(n_img):
        d, patch, found = push.decode_keys(keys[i].cpu())
        m = mm[i]
        assert np.array_equal(m, pu.class_patch_bitmask_fast(labels[i], h, w))
        xd = x[i].double().reshape(C, -1).t()
        exact = (torch.cdist(xd, protos.double()) ** 2).numpy()  # [h*w, P]
        norm = (xd ** 2).sum(1).numpy()[:, None] + (protos.double() ** 2).sum(1).numpy()[None, :]
        for j in range(P):
            member = ((m >> int(pc[j])) & 1).astype(bool)
            if not member.any():
                assert not bool(found[j])
                continue
            q = int(patch[j])
            assert member[q]
            rows = np.nonzero(member)[0]
            cand = exact[rows, j]
            order = np.argsort(cand, kind="stable")
            best = cand[order[0]]
            tol = 2e-6 * norm[member, j].max() + 1e-5 * (1 + best)
            assert exact[q, j] <= best + 2 * tol
            assert abs(float(d[j]) - exact[q, j]) <= tol
            if len(cand) == 1 or cand[order[1]] - best > 2 * tol:
                assert q == int(rows[order[0]]), (i, j, q, int(rows[order[0]]))
                exact_idx += 1
    assert exact_idx > 0


@pytest.mark.parametrize("C,P,n_img,h,w", [(64, 190, 3, 33, 47), (128, 300, 2, 20, 31), (32, 520, 1, 65, 65),
                                           (64, 19, 4, 7, 9)])
def test_push_top2_keys_vs_brute_force(device, C, P, n_img, h, w):
    """Per image: the best key and the runner-up distance (another class patch) against a float64
    brute force of the masked distances; prototype chunks of 8 tiles (P > 256), C = 32 / 128,
    maps smaller than one 128-pixel block."""
    push = _push()
    K = 19
    gen = torch.Generator().manual_seed(C + P)
    x = torch.sigmoid(2 * torch.randn(n_img, C, h, w, generator=gen))
    protos = torch.rand(P, C, generator=gen)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32)
    pc[::7] = -1  # never pushed
    rng = np.random.default_rng(P)
    labels = rng.integers(0, K + 1, size=(n_img, 4 * h, 4 * w)).astype(np.int64)
    mask = push.patch_class_mask(torch.from_numpy(labels).to(device), h, w)
    keys, second = push.push_argmin(x.to(device), protos.to(device), pc.to(device), mask, with_second=True)
    m = mask.cpu().numpy().view(np.uint32)
    for i in range(n_img):
        d1, q1, f1 = push.decode_keys(keys[i].cpu())
        d2, q2, f2 = push.decode_keys(second[i].cpu())
        xd = x[i].double().reshape(C, -1).t()
        exact = (torch.cdist(xd, protos.double()) ** 2).numpy()
        norm = (xd ** 2).sum(1).numpy()[:, None] + (protos.double() ** 2).sum(1).numpy()[None, :]
        for j in range(P):
            member = ((m[i] >> max(int(pc[j]), 0)) & 1).astype(bool) if pc[j] >= 0 else np.zeros(h * w, bool)
            n_member = int(member.sum())
            assert bool(f1[j]) == (n_member >= 1) and bool(f2[j]) == (n_member >= 2), (i, j)
            if n_member == 0:
                continue
            tol = 2e-6 * norm[member, j].max() + 1e-5
            srt = np.sort(exact[member, j])
            assert member[int(q1[j])] and abs(float(d1[j]) - exact[int(q1[j]), j]) <= tol
            assert exact[int(q1[j]), j] <= srt[0] + 2 * tol
            if n_member >= 2:  # runner-up distance (its patch bits are all ones)
                assert int(q2[j]) == 0xFFFFFFFF
                assert abs(float(d2[j]) - srt[1]) <= 2 * tol
                assert float(d2[j]) >= float(d1[j])


@pytest.mark.parametrize("C,P,n_img,h,w", [(64, 190, 8, 129, 257), (64, 361, 3, 65, 65), (32, 520, 2, 33, 47),
                                           (64, 19, 1, 7, 9), (64, 190, 1, 129, 257)])
def test_push_argmin_exact_in_its_own_arithmetic(device, C, P, n_img, h, w):
    """The argmin kernel and protoseg_push_distances (the distances the host re-resolves exact ties
    with) use the same arithmetic bit for bit: each key's distance is push_distances' value at the
    key's patch, no class patch has a smaller one, an equal one only at a higher patch index, and
    the runner-up is the second smallest of push_distances over the class patches (another patch).
    Full Cityscapes-sized maps included, one and eight images per call."""
    push = _push()
    K = 19
    gen = torch.Generator().manual_seed(C * 7 + P)
    x = torch.sigmoid(2 * torch.randn(n_img, C, h, w, generator=gen)).to(device)
    protos = torch.rand(P, C, generator=gen).to(device)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32)
    pc[::5] = -1
    rng = np.random.default_rng(P + h)
    labels = rng.integers(0, K + 1, size=(n_img, 4 * h, 4 * w)).astype(np.int64)
    mask = push.patch_class_mask(torch.from_numpy(labels).to(device), h, w)
    keys, second = push.push_argmin(x, protos, pc.to(device), mask, with_second=True)
    torch.cuda.synchronize()
    mm = mask.cpu().numpy().view(np.uint32)
    pcn = pc.numpy()
    checked = 0
    for i in range(n_img):
        d = push.push_distances(x[i], protos).cpu().numpy()  # [P, h*w] in the argmin's arithmetic
        kd, kp, found = (t.numpy() for t in push.decode_keys(keys[i].cpu()))
        sd, _, sfound = (t.numpy() for t in push.decode_keys(second[i].cpu()))
        for j in range(P):
            if pcn[j] < 0:
                assert not bool(found[j])
                continue
            member = ((mm[i] >> int(pcn[j])) & 1).astype(bool)
            if not member.any():
                assert not bool(found[j])
                continue
            rows = np.nonzero(member)[0]
            vals = d[j, rows]
            q = int(kp[j])
            assert member[q] and np.float32(kd[j]) == d[j, q], (i, j)
            assert vals.min() == d[j, q] and q == int(rows[np.argmin(vals)]), (i, j)  # first index of the minimum
            if len(rows) > 1:
                srt = np.sort(vals)
                assert bool(sfound[j]) and np.float32(sd[j]) == srt[1], (i, j)
            checked += 1
    assert checked > 0


def test_near_tie_flag_fires_on_constructed_ties(device):
    """Exact ties built into the data: (a) a winning patch's feature vector copied to another
    patch of the same class in the same image, (b) a second image identical to the first
    (cross-image tie: strict '<' keeps image 0). near_ties flags exactly the tied prototypes."""
    push = _push()
    C, h, w, P, K = 64, 12, 14, 38, 19
    gen = torch.Generator().manual_seed(5)
    x = torch.sigmoid(2 * torch.randn(1, C, h, w, generator=gen))
    protos = torch.rand(P, C, generator=gen)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32)
    labels = torch.from_numpy(np.repeat(np.repeat(np.random.default_rng(9).integers(1, K + 1, size=(h, w)), 4, 0),
                                        4, 1).astype(np.int64))
    lab = labels.to(device)
    st = push.PushState.create(P, C, device)
    push.push_update(st, x.to(device), lab, protos.to(device), pc.to(device), 0)
    base_flags = push.near_ties(st, protos)
    # (a) duplicate prototype 3's winning patch at another patch of its class
    j = 3
    q = int(st.patch[j])
    small = labels.reshape(h, 4, w, 4)[:, 0, :, 0].reshape(-1)
    same = [int(t) for t in np.nonzero(small.numpy() == small[q].item())[0] if t != q]
    assert same, "test setup: the class of the winning patch has another patch"
    x2 = x.clone()
    x2.view(1, C, -1)[0, :, same[0]] = x.view(1, C, -1)[0, :, q]
    st2 = push.PushState.create(P, C, device)
    push.push_update(st2, x2.to(device), lab, protos.to(device), pc.to(device), 0)
    flags = push.near_ties(st2, protos)
    assert j in flags
    assert int(st2.patch[j]) == min(q, same[0])  # the kernel's own pick: the lower patch index
    assert float(st2.second[j]) == float(st2.dist[j])
    assert j in push.exact_tie_candidates(st2)
    # resolved in the reference's order: the oracle's literal loop (list(set) + np.argmin)
    push.resolve_exact_ties(st2, lambda i: (x2.to(device), lab), protos.to(device), pc)
    ost = pu.PushOracleState(P, C)
    d = po.l2_convolution(x2, protos[:, :, None, None], torch.ones(P, C, 1, 1))[0]
    assert d.reshape(P, -1)[j, q] == d.reshape(P, -1)[j, same[0]]
    pu.update_prototypes_on_image_core(ost, x2[0].numpy(), d.permute(1, 2, 0).numpy(), labels.numpy(), pc.numpy(),
                                       K, 0)
    assert int(st2.patch[j]) == int(ost.winner_patch[j])
    assert torch.equal(st2.fmap[j].cpu(), x2.view(C, -1)[:, int(ost.winner_patch[j])])
    # (b) the same image twice: every found prototype ties across images, image 0 wins
    st3 = push.PushState.create(P, C, device)
    push.push_update(st3, torch.cat([x, x]).to(device), torch.stack([lab, lab]), protos.to(device), pc.to(device), 0)
    found = np.nonzero(st3.img.cpu().numpy() >= 0)[0]
    assert len(found) > 0 and set(found) <= set(push.near_ties(st3, protos))
    assert (st3.img.cpu().numpy()[found] == 0).all()
    # flags of the untouched scan are only genuine near-ties: the gap is within the band
    band = 1e-5 * ((st.fmap.cpu() ** 2).sum(1) + (protos ** 2).sum(1))
    gap = (st.second - st.dist).cpu()
    for k in range(P):
        assert (k in base_flags) == bool(st.img[k] >= 0 and gap[k] <= band[k])


def test_exact_ties_resolve_in_reference_order_golden(device):
    """push_ties.npz (3 images, every minimum shared by several patches, equal minima across
    images): kernel scan + resolve_exact_ties equals the oracle's literal push.py loop in every
    winning image, patch, distance, feature vector and rf box."""
    push = _push()
    g = np.load(os.path.join(GOLDEN, "push_ties.npz"))
    x = torch.from_numpy(g["x"]).to(device)
    protos = torch.from_numpy(g["protos"]).to(device)
    pc = torch.from_numpy(g["proto_class"]).to(device)
    labels = torch.from_numpy(g["labels"]).to(device)
    P, C = protos.shape
    for per in (1, 3):  # one image per call (the drop-in) and the batched scan
        state = push.PushState.create(P, C, device)
        for i0 in range(0, x.shape[0], per):
            push.push_update(state, x[i0:i0 + per], labels[i0:i0 + per], protos, pc, i0)
        cand = push.exact_tie_candidates(state)
        assert len(cand) == P  # every prototype holds a tie at its minimum
        moved = push.resolve_exact_ties(state, lambda i: (x[i:i + 1], labels[i]), protos, pc)
        assert len(moved) > 0
        assert np.array_equal(state.img.cpu().numpy(), g["proto_rf_boxes"][:, 0])
        assert np.array_equal(state.patch.cpu().numpy(), g["winner_patch"])
        assert np.array_equal(push.rf_boxes(state, g["proto_class"]), g["proto_rf_boxes"])
        assert np.array_equal(state.fmap.cpu().numpy(), g["global_min_fmap_patches"].astype(np.float32))
        assert np.allclose(state.dist.cpu().numpy(), g["global_min_proto_dist"], rtol=1e-5, atol=1e-5)


def test_push_distances_equal_the_argmin_kernel(device):
    """push_distances reproduces push_argmin's keys bit for bit (same arithmetic)."""
    push = _push()
    C, h, w, P, K = 64, 33, 47, 57, 19
    gen = torch.Generator().manual_seed(77)
    x = torch.sigmoid(2 * torch.randn(1, C, h, w, generator=gen)).to(device)
    protos = torch.rand(P, C, generator=gen).to(device)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32).to(device)
    labels = torch.from_numpy(np.random.default_rng(1).integers(0, K + 1, size=(4 * h, 4 * w))).to(device)
    mask = push.patch_class_mask(labels, h, w)
    keys = push.push_argmin(x, protos, pc, mask)
    dk, qk, fk = push.decode_keys(keys[0].cpu())
    d = push.push_distances(x, protos).cpu()
    m = mask.cpu().numpy().view(np.uint32)[0]
    for j in range(P):
        member = torch.from_numpy(((m >> int(pc[j])) & 1).astype(bool))
        if not member.any():
            continue
        dj = torch.where(member, d[j], torch.tensor(float("inf")))
        assert float(dj.min()) == float(dk[j])
        assert int(torch.nonzero(dj == dj.min())[0]) == int(qk[j])


def test_push_prototypes_batched_scan_resolves_planted_ties(device, tmp_path):
    """push_prototypes at images_per_batch = 8 with a backbone whose features depend on the batch
    shape (as batched convolutions may, bit for bit) and quantised so that every class minimum is
    an exact tie of several patches: the tie resolution recomputes each winning image in its scan
    batch, so every tie is reproduced (no 'not reproduced' log line) and the winners equal the
    reference loop (oracle push.py:195-307, list(set) order) on the features the scan used."""
    import torch.nn.functional as F
    from PIL import Image

    from oracle import push_oracle as pu
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    from protoseg_amd.model import PPNet
    from protoseg_amd.push import push_prototypes

    push = _push()
    torch.manual_seed(0)
    P, K, C = 38, 19, 64
    net = PPNet(deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[]), 513, (P, C, 1, 1), None, K,
                add_on_layers_type="deeplab_simple").to(device).eval()
    proj = (torch.randint(-4, 5, (C, 3), generator=torch.Generator().manual_seed(2)).float() / 8).to(device)

    def fake_features(imgs):
        q = torch.round(F.avg_pool2d(imgs, 8) * 2) / 2  # few distinct patches: exact ties
        f = torch.sigmoid(torch.einsum("oc,nchw->nohw", proj, q))
        return f + 1e-3 * imgs.shape[0]  # batch-shape dependent, like a batched convolution

    net.conv_features = fake_features
    rng = np.random.default_rng(5)
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
        np.save(ann_dir / f"{img_id}.npy", rng.integers(0, K + 1, size=(64, 96)).astype(np.int64))
    protos0 = net.prototype_vectors.detach().reshape(P, C).clone()  # the push projects and prunes them
    pc = push.prototype_classes(net).cpu().numpy()
    logs = []
    state = push_prototypes(ds, net, images_per_batch=8, log=lambda *a: logs.append(" ".join(map(str, a))))
    assert not any("not reproduced" in line for line in logs), logs
    assert any("exact tie(s) resolved" in line for line in logs)

    # the reference loop on the scan's features (one backbone batch of the three images)
    from protoseg_amd.push import to_normalized_tensor
    with torch.no_grad():
        imgs = torch.cat([to_normalized_tensor(Image.open(ds.get_img_path(i)).convert("RGB").crop((4, 4, 100, 68)))
                          .unsqueeze(0) for i in ds.img_ids]).to(device)
        feats = fake_features(imgs)
    ref = pu.PushOracleState(P, C)
    for i, img_id in enumerate(ds.img_ids):
        d = push.push_distances(feats[i:i + 1], protos0).cpu().numpy()  # [P, h*w]
        h, w = feats.shape[2:]
        y = np.load(ann_dir / f"{img_id}.npy")
        pu.update_prototypes_on_image_core(ref, feats[i].cpu().numpy(), d.reshape(P, h, w).transpose(1, 2, 0), y, pc,
                                           K, i)
    found = ref.proto_rf_boxes[:, 0] >= 0
    assert found.sum() > 10
    assert np.array_equal(state.img.cpu().numpy(), ref.proto_rf_boxes[:, 0])
    assert np.array_equal(state.patch.cpu().numpy()[found], ref.winner_patch[found])


def test_push_update_one_call_equals_three_calls(device):
    """protoseg_push_update (one host call, masks / keys in library scratch) leaves the state the
    mask -> argmin -> merge sequence leaves, bit for bit, over two batches."""
    from protoseg_amd import _lib
    push = _push()
    C, h, w, P, K, n = 64, 17, 23, 40, 19, 3
    gen = torch.Generator().manual_seed(21)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32).to(device)
    protos = torch.rand(P, C, generator=gen).to(device)
    a, b = push.PushState.create(P, C, device), push.PushState.create(P, C, device)
    for first in (0, n):
        x = torch.sigmoid(2 * torch.randn(n, C, h, w, generator=gen)).to(device)
        lab = torch.from_numpy(np.random.default_rng(first).integers(0, K + 1, size=(n, 4 * h, 4 * w))).to(device)
        push.push_update(a, x, lab, protos, pc, first)
        mask = push.patch_class_mask(lab, h, w)
        keys, second = push.push_argmin(x, protos, pc, mask, with_second=True)
        if b.second is None:
            b.second = torch.full((P,), float("inf"), device=device)
        with torch.cuda.device(device):
            _lib.call("protoseg_push_merge", _lib.ptr(keys), _lib.ptr(second), n, first, _lib.ptr(x), C, h * w, P,
                      _lib.ptr(b.dist), _lib.ptr(b.second), _lib.ptr(b.img), _lib.ptr(b.patch), _lib.ptr(b.fmap),
                      _lib.stream_of(device))
    torch.cuda.synchronize()
    for f in ("dist", "second", "img", "patch", "fmap"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize("P", [40, 190, 361])
def test_push_update_scan_bound_keeps_state(device, P):
    """A scan of many batches through protoseg_push_update, whose argmin skips candidates above
    the running runner-up (push_argmin_wave_kernel's bound), leaves the same state bit for bit as
    the unbounded mask -> argmin -> merge sequence: best distance, runner-up, image, patch and
    winning feature vector. Later batches are pruned almost entirely (the bound is tight), and
    one batch repeats an earlier image exactly, so exact cross-image ties meet the bound too."""
    from protoseg_amd import _lib
    push = _push()
    C, h, w, K, n = 64, 33, 65, 19, 4
    gen = torch.Generator().manual_seed(5)
    pc = torch.argmax(po.class_identity(P, K), dim=1).to(torch.int32).to(device)
    protos = torch.rand(P, C, generator=gen).to(device)
    a, b = push.PushState.create(P, C, device), push.PushState.create(P, C, device)
    xs = []
    for bi in range(8):
        x = torch.sigmoid(2 * torch.randn(n, C, h, w, generator=gen)).to(device)
        if bi == 5:
            x[1] = xs[0][2]  # an exact repeat of an earlier image: ties at the running best
        xs.append(x)
        lab = torch.from_numpy(np.random.default_rng(bi).integers(0, K + 1, size=(n, 4 * h, 4 * w))).to(device)
        if bi == 5:
            lab[1] = torch.from_numpy(np.random.default_rng(0).integers(0, K + 1, size=(n, 4 * h, 4 * w))[2]).to(device)
        first = bi * n
        push.push_update(a, x, lab, protos, pc, first)
        mask = push.patch_class_mask(lab, h, w)
        keys, second = push.push_argmin(x, protos, pc, mask, with_second=True)
        with torch.cuda.device(device):
            _lib.call("protoseg_push_merge", _lib.ptr(keys), _lib.ptr(second), n, first, _lib.ptr(x), C, h * w, P,
                      _lib.ptr(b.dist), _lib.ptr(b.second), _lib.ptr(b.img), _lib.ptr(b.patch), _lib.ptr(b.fmap),
                      _lib.stream_of(device))
    torch.cuda.synchronize()
    for f in ("dist", "second", "img", "patch", "fmap"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    assert (a.img >= 0).all()


def test_push_prototypes_kxk_prototypes(device, tmp_path):
    """push_prototypes with 2 x 2 prototypes (push.py:276-280 keeps the k x k window
    protoL_input_[:, i:i+h, j:j+w]): the scan runs on the unfolded map; winners, patches and the
    pushed windows equal the reference loop (oracle push.py:195-307) on the same windows."""
    from PIL import Image

    from oracle import push_oracle as pu
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    from protoseg_amd.model import PPNet
    from protoseg_amd.push import push_prototypes, to_normalized_tensor

    push = _push()
    torch.manual_seed(1)
    P, K, C, k = 38, 19, 64, 2
    net = PPNet(deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[]), 513, (P, C, k, k), None, K,
                add_on_layers_type="deeplab_simple").to(device).eval()
    proj = torch.randn(C, 3, generator=torch.Generator().manual_seed(4)).to(device)
    # an elementwise stand-in backbone: bit-reproducible across calls and batch compositions
    net.conv_features = lambda imgs: torch.sigmoid(torch.einsum("oc,nchw->nohw", proj,
                                                                torch.nn.functional.avg_pool2d(imgs, 8)))
    rng = np.random.default_rng(3)
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
        np.save(ann_dir / f"{img_id}.npy", rng.integers(0, K + 1, size=(64, 96)).astype(np.int64))
    protos0 = net.prototype_vectors.detach().reshape(P, -1).clone()
    pc = push.prototype_classes(net).cpu().numpy()
    with torch.no_grad():
        imgs = torch.cat([to_normalized_tensor(Image.open(ds.get_img_path(i)).convert("RGB").crop((4, 4, 100, 68)))
                          .unsqueeze(0) for i in ds.img_ids]).to(device)
        f = net.conv_features(imgs)
        n, c, H, W = f.shape
        feats = torch.nn.functional.unfold(f, (k, k)).reshape(n, c * k * k, H - k + 1, W - k + 1)
    state = push_prototypes(ds, net, images_per_batch=8, log=lambda *_: None)
    ref = pu.PushOracleState(P, C * k * k)
    h, w = feats.shape[2:]
    for i, img_id in enumerate(ds.img_ids):
        d = push.push_distances(feats[i:i + 1], protos0).cpu().numpy()
        pu.update_prototypes_on_image_core(ref, feats[i].cpu().numpy(), d.reshape(P, h, w).transpose(1, 2, 0),
                                           np.load(ann_dir / f"{img_id}.npy"), pc, K, i)
    found = ref.proto_rf_boxes[:, 0] >= 0
    assert found.sum() > 10
    assert np.array_equal(state.img.cpu().numpy(), ref.proto_rf_boxes[:, 0])
    assert np.array_equal(state.patch.cpu().numpy()[found], ref.winner_patch[found])
    assert np.array_equal(state.fmap.cpu().numpy()[found],
                          ref.global_min_fmap_patches.reshape(P, -1)[found].astype(np.float32))
    assert tuple(net.prototype_vectors.shape[1:]) == (C, k, k)  # pushed windows keep the k x k shape
