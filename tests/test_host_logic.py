"""CPU: host-side logic of the PPNet mirror and the push driver (no kernel calls)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import push_oracle as pu
from protoseg_amd import ProtosegError
from protoseg_amd.deeplab import deeplabv2_resnet101_features
from protoseg_amd.distributed import shard_bounds
from protoseg_amd.model import PPNet, construct_PPNet
from protoseg_amd import push as dpush


def small_ppnet(P=38, K=19):
    feats = deeplabv2_resnet101_features(n_blocks=(1, 1, 1, 1), scales=[])
    return PPNet(feats, 513, (P, 64, 1, 1), None, K, add_on_layers_type="deeplab_simple", patch_classification=True)


def test_ppnet_surface_matches_reference():
    net = small_ppnet()
    assert net.prototype_shape == torch.Size([38, 64, 1, 1])
    assert net.num_prototypes == 38 and net.num_classes == 19 and net.num_prototypes_per_class == 2
    assert net.epsilon == 1e-4
    assert net.prototype_class_identity.shape == (38, 19)
    assert torch.equal(net.prototype_class_identity.argmax(1), torch.arange(38) // 2)
    assert not net.ones.requires_grad and net.prototype_vectors.requires_grad
    assert net.last_layer.bias is None
    w = net.last_layer.weight
    assert torch.all((w == 1) | (w == -0.5)) and torch.all(w.sum(1) == 2 * 1 + 36 * -0.5)
    for name in ("c0", "c1", "c2", "c3"):
        assert hasattr(net.features.base.aspp, name)
    net.features.base.freeze_bn()
    assert isinstance(net.add_on_layers[0], torch.nn.Sigmoid)
    assert str(net).startswith("PPNet(")


def test_construct_ppnet_full_backbone_shapes():
    net = construct_PPNet(img_size=513, pretrained=False, prototype_shape=(190, 64, 1, 1), num_classes=19,
                          add_on_layers_type="deeplab_simple")
    net.eval()
    with torch.no_grad():
        feats = net.conv_features(torch.zeros(1, 3, 513, 513))
    assert feats.shape == (1, 64, 65, 65)  # output stride 8, ceil-mode pool (push.py:275)
    assert net.proto_layer_rf_info == [513, 1, 1, 0.5]
    with pytest.raises(ProtosegError):
        construct_PPNet(base_architecture="vgg16", pretrained=False)


def test_prune_prototypes():
    net = small_ppnet()
    w_before = net.last_layer.weight.data.clone()
    net.prune_prototypes([0, 5, 37])
    assert net.num_prototypes == 35
    keep = [i for i in range(38) if i not in (0, 5, 37)]
    assert torch.equal(net.last_layer.weight.data, w_before[:, keep])
    assert net.last_layer.in_features == 35
    assert net.ones.shape[0] == 35 and net.prototype_class_identity.shape == (35, 19)


def test_cpu_forward_fails_loudly():
    net = small_ppnet()
    with pytest.raises((ProtosegError, RuntimeError, NotImplementedError)):
        net.forward_from_conv_features(torch.rand(1, 64, 3, 3))


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 2975):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_lut_from_convert_targets():
    conv = np.vectorize(pu.CITYSCAPES_19_EVAL_CATEGORIES.get)
    lut = dpush.lut_from_convert_targets(conv)
    raw = np.random.default_rng(0).integers(0, 29, size=(50, 60))
    assert np.array_equal(lut[raw], conv(raw))
    assert dpush.lut_from_convert_targets(None) is None


def test_rf_boxes_match_reference_formula():
    P = 4
    state = dpush.PushState.create(P, 8, "cpu")
    state.img[:] = torch.tensor([0, 3, -1, 3])
    state.patch[:] = torch.tensor([0, 257 * 128 + 256, -1, 1000], dtype=torch.int32)
    state.geometry = {0: (1024, 2048, 129, 257), 3: (1024, 2048, 129, 257)}
    boxes = dpush.rf_boxes(state, np.array([0, 1, 2, 3]))
    ph, pw = 1024 / 129, 2048 / 257
    for j, (img, patch) in enumerate([(0, 0), (3, 257 * 128 + 256), (None, None), (3, 1000)]):
        if img is None:
            assert (boxes[j] == -1).all()
            continue
        i, jj = divmod(patch, 257)
        assert list(boxes[j]) == [img, int(i * ph), int(i * ph + ph) + 1, int(jj * pw), int(jj * pw + pw) + 1, j]


def test_dedup_and_prune(tmp_path):
    net = small_ppnet(P=6, K=3)
    fmap = np.random.default_rng(1).random((6, 64)).astype(np.float32)
    fmap[4] = fmap[1]          # a duplicate pushed prototype
    fmap[5] = 0                # never pushed (stays zero) ...
    fmap[3] = 0                # ... twice: only the first zero row survives
    dup = dpush.dedup_and_prune(net, fmap, str(tmp_path), log=lambda *_: None)
    uniq, ref_dup = pu.dedup(fmap.astype(np.float64))
    assert dup == ref_dup == [4, 5]
    assert json.load(open(os.path.join(tmp_path, "unique_prototypes.json"))) == sorted(int(i) for i in uniq)
    assert net.num_prototypes == 4
