"""Generates the committed golden vectors from the oracle (CPU restatement of the reference).

The reference repository ships no tests or fixtures for this path and its Python cannot be
run here, so these vectors freeze the oracle's outputs on seeded inputs;
tests/test_oracle.py re-derives them bit for bit and the GPU tests compare the HIP kernels
against them. Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import protoseg_oracle as po  # noqa: E402
from oracle import kld_oracle as ko  # noqa: E402
from oracle import push_oracle as pu  # noqa: E402
from oracle import knn_oracle as kn  # noqa: E402
from oracle import bbox_oracle as bo  # noqa: E402

SEED = 20220227


def l2_case(B, C, h, w, P, K, seed):
    x, protos, w_last = po.synthetic_inputs(B, C, h, w, P, K, seed)
    gen = torch.Generator().manual_seed(seed + 1)
    # a trained-looking last layer: identity init plus noise
    w_last = w_last + 0.1 * torch.randn(w_last.shape, generator=gen)
    g_logits = torch.randn(B, h, w, K, generator=gen)
    g_dist = 0.01 * torch.randn(B, P, h, w, generator=gen)
    logits, dist, gx, gp, gw = po.forward_backward(x, protos, w_last, g_logits, None)
    _, _, gx_d, gp_d, _ = po.forward_backward(x, protos, w_last, g_logits, g_dist)
    _, act = po.forward_from_conv_features(x, protos[:, :, None, None], w_last, return_activations=True)
    return dict(x=x.numpy(), protos=protos.numpy(), w_last=w_last.numpy(), g_logits=g_logits.numpy(),
                g_dist=g_dist.numpy(), logits=logits.numpy(), dist=dist.numpy(), act=act.detach().numpy(),
                g_x=gx.numpy(), g_protos=gp.numpy(), g_w=gw.numpy(), g_x_with_gdist=gx_d.numpy(),
                g_protos_with_gdist=gp_d.numpy())


def push_case(n_img, C, H, W, h, w, P, K, seed):
    rng = np.random.default_rng(seed)
    gen = torch.Generator().manual_seed(seed)
    x = torch.sigmoid(2.0 * torch.randn(n_img, C, h, w, generator=gen))
    protos = torch.rand(P, C, generator=gen)
    identity = po.class_identity(P, K)
    proto_class = torch.argmax(identity, dim=1).numpy().astype(np.int32)
    # raw Cityscapes ids 0..28 in blocks, so classes cover contiguous regions
    raw = rng.integers(0, 29, size=(n_img, H // 4, W // 4))
    raw = np.repeat(np.repeat(raw, 4, axis=1), 4, axis=2)[:, :H, :W].astype(np.int64)
    labels = np.stack([pu.convert_targets(r) for r in raw]).astype(np.int64)
    state = pu.PushOracleState(P, C)
    dists, masks = [], []
    for i in range(n_img):
        d = po.l2_convolution(x[i:i + 1], protos[:, :, None, None], torch.ones(P, C, 1, 1))[0]
        proto_dist_ = d.permute(1, 2, 0).numpy()
        sets = pu.class_to_patch_index_dict(labels[i], h, w, K)
        masks.append(pu.bitmask_from_dict(sets, h, w))
        pu.update_prototypes_on_image_core(state, x[i].numpy(), proto_dist_, labels[i], proto_class, K, i, sets)
        dists.append(d.numpy())
    unique_index, duplicate_idx = pu.dedup(state.global_min_fmap_patches.reshape(P, C, 1, 1))
    return dict(x=x.numpy(), protos=protos.numpy(), proto_class=proto_class, raw_labels=raw, labels=labels,
                dist=np.stack(dists), mask=np.stack(masks), global_min_proto_dist=state.global_min_proto_dist,
                global_min_fmap_patches=state.global_min_fmap_patches.reshape(P, C), winner_patch=state.winner_patch,
                proto_rf_boxes=state.proto_rf_boxes, unique_index=np.asarray(unique_index),
                duplicate_idx=np.asarray(duplicate_idx, dtype=np.int64))


def push_ties_case(n_img, C, H, W, h, w, P, K, n_vec, seed):
    """push.py:184-281 where exact ties inside an image are the rule: every patch of an image
    carries one of ``n_vec`` feature vectors, so each prototype's class minimum is shared by
    many patches and np.argmin over the list(set) order of push.py:214-230 picks the winner.
    Images 0 and 2 share their vector table (equal minima across images: strict '<' keeps image
    0); the labels differ, so the set orders differ."""
    rng = np.random.default_rng(seed)
    gen = torch.Generator().manual_seed(seed)
    tables = torch.sigmoid(2.0 * torch.randn(2, C, n_vec, generator=gen))
    xs = []
    for i in range(n_img):
        pick = torch.from_numpy(rng.integers(0, n_vec, size=h * w))
        xs.append(tables[i % 2][:, pick].reshape(C, h, w))
    x = torch.stack(xs)
    protos = torch.rand(P, C, generator=gen)
    proto_class = torch.argmax(po.class_identity(P, K), dim=1).numpy().astype(np.int32)
    # class regions in blocks of 3 pixels: not aligned with the 8x8 patches, so patches hold
    # several classes and each class's set is built in an order that is not the patch order
    y = rng.integers(0, K + 1, size=(n_img, H // 3 + 1, W // 3 + 1))
    labels = np.repeat(np.repeat(y, 3, axis=1), 3, axis=2)[:, :H, :W].astype(np.int64)
    state = pu.PushOracleState(P, C)
    dists, masks = [], []
    for i in range(n_img):
        d = po.l2_convolution(x[i:i + 1], protos[:, :, None, None], torch.ones(P, C, 1, 1))[0]
        # equal feature vectors must give equal distances in the oracle's arithmetic
        flat = d.reshape(P, -1).numpy()
        vec = x[i].reshape(C, -1).numpy()
        for q in range(1, h * w):
            same = np.nonzero((vec[:, :q] == vec[:, q:q + 1]).all(0))[0]
            if same.size:
                assert np.array_equal(flat[:, same[0]], flat[:, q])
        sets = pu.class_to_patch_index_dict(labels[i], h, w, K)
        masks.append(pu.bitmask_from_dict(sets, h, w))
        pu.update_prototypes_on_image_core(state, x[i].numpy(), d.permute(1, 2, 0).numpy(), labels[i], proto_class, K,
                                           i, sets)
        dists.append(d.numpy())
    return dict(x=x.numpy(), protos=protos.numpy(), proto_class=proto_class, labels=labels, dist=np.stack(dists),
                mask=np.stack(masks), global_min_proto_dist=state.global_min_proto_dist,
                global_min_fmap_patches=state.global_min_fmap_patches.reshape(P, C), winner_patch=state.winner_patch,
                proto_rf_boxes=state.proto_rf_boxes)


def kld_case(B, h, w, P, K, seed):
    """module.py:167-208 on the distances of a trained-looking layer: labels in blocks with
    void, every class value and the skipped value K present; one class with a single pixel."""
    x, protos, _ = po.synthetic_inputs(B, 64, h, w, P, K, seed)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, 64, 1, 1))
    target = ko.synthetic_targets(B, h, w, K, seed + 1, block=3)
    absent = [c for c in range(1, K) if int((target[1] == c).sum()) == 0]
    if absent:
        target[1, 0] = absent[0]  # a class with a single pixel: no distribution (module.py:186)
    identity = po.class_identity(P, K)
    loss, n_pairs, g_dist = ko.kld_loss_and_grad(dist, target, identity, g_loss=1.0)
    return dict(dist=dist.numpy(), target=target.numpy(), proto_class=torch.argmax(identity, 1).numpy().astype(np.int32),
                num_classes=np.int64(K), loss=np.float32(loss), n_pairs=np.int64(n_pairs), g_dist=g_dist.numpy())


def knn_case(n_img, C, H, W, h, w, P, K, k, seed):
    """find_nearest.py:87-232 + prune.py:35-43 on l2 distance maps of seeded features; image 4
    is all void (the 10e6 mask decides alone), image 5 repeats image 1 (exact ties across
    images: heapq keeps the earlier one)."""
    dists = []
    for i in range(n_img):
        x, protos, _ = po.synthetic_inputs(1, C, h, w, P, K, seed)  # same prototypes every image
        x = po.synthetic_inputs(1, C, h, w, P, K, seed + 100 + i)[0]
        dists.append(po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, C, 1, 1))[0].numpy())
    _, labels = kn.synthetic_search(n_img, 1, 1, 1, H, W, K, seed + 1)
    labels[4][:] = 0
    dists[5] = dists[1].copy()
    labels[5] = labels[1].copy()
    proto_class = (np.arange(P) * K // P).astype(np.int32)
    res = kn.find_k_nearest(dists, [y - 1 for y in labels], proto_class, k)
    pruned = kn.prune_list(res["label"], proto_class, 3)
    return dict(dist=np.stack(dists), labels=np.stack(labels), proto_class=proto_class, k=np.int64(k),
                prune_threshold=np.int64(3), out_dist=res["dist"], out_label=res["label"], out_img=res["img"],
                out_patch=res["patch"], pruned=np.array(pruned, np.int64))


def bbox_case(m, C, H, W, h, w, P, K, seed):
    """push.py:309-329 + helpers.py:48-82 for m prototypes on one image: l2 distances of seeded
    features, activation, INTER_CUBIC restatement, np.percentile(95), gt-class greedy crop."""
    x, protos, _ = po.synthetic_inputs(1, C, h, w, P, K, seed)
    dist = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, C, 1, 1))[0].numpy()[:m]
    rng = np.random.default_rng(seed)
    y = rng.integers(0, K + 1, size=(H // 8, W // 8))
    y = np.repeat(np.repeat(y, 8, 0), 8, 1).astype(np.int64)
    proto_class = (np.arange(m) * K // m).astype(np.int32)
    rf = np.zeros((m, 4), np.int64)
    thr = np.zeros(m, np.float32)
    box = np.zeros((m, 4), np.int64)
    up = np.zeros((m, H, W), np.float32)
    for j in range(m):
        i0, j0 = np.unravel_index(int(np.argmin(dist[j])), dist[j].shape)
        rf[j] = bo.rf_box(int(i0), int(j0), H, W, h, w)
        t, b, u = bo.bound_box(dist[j], y, int(proto_class[j]), rf[j], "log", 1e-4, C)
        thr[j], box[j], up[j] = t, b, u
    return dict(dist=dist, labels=y, proto_class=proto_class, rf=rf, up=up, threshold=thr, box=box)


CASES = {
    "l2_small": lambda: l2_case(2, 64, 17, 17, 38, 19, SEED),
    "l2_ragged": lambda: l2_case(3, 32, 7, 11, 21, 3, SEED + 7),
    "push_small": lambda: push_case(3, 64, 64, 128, 8, 16, 38, 19, SEED),
    "push_ties": lambda: push_ties_case(3, 64, 64, 128, 8, 16, 38, 19, 6, SEED + 3),
    "kld_small": lambda: kld_case(2, 13, 17, 38, 19, SEED + 11),
    "knn_small": lambda: knn_case(7, 32, 60, 110, 9, 13, 38, 4, 5, SEED + 13),
    "bbox_small": lambda: bbox_case(6, 64, 72, 136, 9, 17, 38, 19, SEED + 17),
}


def main(only=None):
    for name, fn in CASES.items():
        if only and name not in only:
            continue
        arrays = fn()
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrays)
        print(f"wrote {path} ({os.path.getsize(path)} B)")


if __name__ == "__main__":
    main(sys.argv[1:])
