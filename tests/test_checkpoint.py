"""Checkpoint compatibility with the reference (segmentation/module.py:292-297,
train.py:60-64, 153, 192-200, eval_valid.py:33): whole-module pickles and reference-keyed state
dicts.

The expected key set is derived independently of this build's modules: the torchvision
ResNet-101 key names (conv1 / bn1, layer1..4 blocks with conv1..3 / bn1..3 and downsample.0/1)
mapped by a restatement of the reference's own remap deeplab_features.py:8-49, prefixed
``features.base.`` (MSC.base, segmentation/utils.py:64-75), plus the ASPP branches
``aspp.c0..c3`` (module.py:336-343) and PPNet's own parameters (model.py:54, 140-144).
"""
import io
import sys
import types

import pytest
import torch
from torch import nn


def _pkg():
    from protoseg_amd import checkpoint, model
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    return checkpoint, model, deeplabv2_resnet101_features


def torchvision_resnet101_keys():
    """torchvision.models.resnet101().state_dict() key names (fc excluded: the remap drops it)."""
    bn = ("weight", "bias", "running_mean", "running_var", "num_batches_tracked")
    keys = ["conv1.weight"] + [f"bn1.{s}" for s in bn]
    for layer, n in zip(range(1, 5), (3, 4, 23, 3)):
        for b in range(n):
            for i in (1, 2, 3):
                keys.append(f"layer{layer}.{b}.conv{i}.weight")
                keys += [f"layer{layer}.{b}.bn{i}.{s}" for s in bn]
            if b == 0:
                keys.append(f"layer{layer}.{b}.downsample.0.weight")
                keys += [f"layer{layer}.{b}.downsample.1.{s}" for s in bn]
    return keys


def reference_remap(key):
    """deeplab_features.py:8-49 (torchvision_resnet_weight_key_to_deeplab2), restated."""
    seg = key.split(".")
    if seg[0].startswith("layer"):
        dl_layer = int(seg[0][len("layer"):]) + 1
        block = f"block{int(seg[1]) + 1}"
        if seg[2] == "downsample":
            return f"layer{dl_layer}.{block}.shortcut.{('conv', 'bn')[int(seg[3])]}.{seg[-1]}"
        kind, num = seg[2][:-1], int(seg[2][-1])
        return f"layer{dl_layer}.{block}.{('reduce', 'conv3x3', 'increase')[num - 1]}.{kind}.{seg[-1]}"
    if seg[0] in ("conv1", "bn1"):
        return f"layer1.conv1.{seg[0][:-1]}.{seg[-1]}"
    return None


def reference_ppnet_keys(n_aspp=4):
    keys = {"features.base." + reference_remap(k) for k in torchvision_resnet101_keys()}
    for i in range(n_aspp):
        keys |= {f"features.base.aspp.c{i}.weight", f"features.base.aspp.c{i}.bias"}
    return keys | {"prototype_vectors", "ones", "last_layer.weight"}  # deeplab_simple: no add-on params


def _ppnet(n_blocks=(3, 4, 23, 3), P=190, K=19):
    _, model, feats = _pkg()
    torch.manual_seed(0)
    return model.construct_PPNet(img_size=513, prototype_shape=(P, 64, 1, 1), num_classes=K,
                                 add_on_layers_type="deeplab_simple", patch_classification=True,
                                 features=feats(pretrained=False, deeplab_n_features=64, scales=[],
                                                n_blocks=n_blocks))


def test_state_dict_keys_are_the_references():
    ppnet = _ppnet()
    sd = ppnet.state_dict()
    assert set(sd) == reference_ppnet_keys()
    assert tuple(sd["features.base.layer1.conv1.conv.weight"].shape) == (64, 3, 7, 7)
    assert tuple(sd["features.base.layer5.block3.increase.bn.running_var"].shape) == (2048,)
    assert tuple(sd["features.base.aspp.c3.weight"].shape) == (64, 2048, 3, 3)
    assert tuple(sd["prototype_vectors"].shape) == (190, 64, 1, 1)
    assert tuple(sd["ones"].shape) == (190, 64, 1, 1)
    assert tuple(sd["last_layer.weight"].shape) == (19, 190)


def test_reference_state_dict_loads_strict():
    checkpoint, _, _ = _pkg()
    ppnet = _ppnet()
    gen = torch.Generator().manual_seed(3)
    ref_sd = {}
    for k, v in ppnet.state_dict().items():  # same keys as reference_ppnet_keys() (test above)
        ref_sd[k] = v.clone() if v.dtype == torch.int64 else torch.rand(v.shape, generator=gen)
    res = checkpoint.load_state_dict_into(ppnet, ref_sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    for k, v in ppnet.state_dict().items():
        assert torch.equal(v, ref_sd[k]), k
    with pytest.raises(ValueError):
        checkpoint.load_state_dict_into(_ppnet((1, 1, 1, 1), P=38), {"prototype_vectors": torch.rand(19, 64, 1, 1)})


def _same_module(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert set(sa) == set(sb)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    assert torch.equal(a.prototype_class_identity, b.prototype_class_identity)
    assert a.epsilon == b.epsilon and a.prototype_activation_function == b.prototype_activation_function
    assert a.num_prototypes_per_class == b.num_prototypes_per_class and a.img_size == b.img_size


def test_whole_module_round_trip():
    """module.py:292 torch.save(obj=ppnet) -> train.py:60 torch.load(path): this build's class."""
    checkpoint, model, _ = _pkg()
    ppnet = _ppnet((1, 1, 1, 1))
    ppnet.prune_prototypes([3, 17])  # a pruned model (model.py:311-336) keeps its shapes
    buf = io.BytesIO()
    checkpoint.save_ppnet(ppnet, buf)
    buf.seek(0)
    back = checkpoint.load_ppnet(buf)
    assert type(back) is model.PPNet
    _same_module(ppnet, back)
    assert back.num_prototypes == 188 and back.last_layer.weight.shape == (19, 188)


def test_reference_written_pickle_loads_through_the_shim(monkeypatch):
    """A checkpoint the reference wrote pickles ``model.PPNet``; INTEGRATION.md's shim makes that
    name this build's class, and the reference's attribute dict drives it unchanged."""
    checkpoint, model, _ = _pkg()
    ours = _ppnet((1, 1, 1, 1))
    fake = types.ModuleType("model")

    class PPNet(nn.Module):  # the reference's class as pickle sees it: model.PPNet, its own __dict__
        pass

    PPNet.__module__, PPNet.__qualname__ = "model", "PPNet"
    fake.PPNet = PPNet
    monkeypatch.setitem(sys.modules, "model", fake)
    ref_obj = PPNet()
    ref_obj.__dict__.update({k: v for k, v in ours.__dict__.items() if k not in ("precision",)})
    buf = io.BytesIO()
    torch.save(ref_obj, buf)
    # the reference's model.py with the shim appended
    fake.PPNet, fake.construct_PPNet = model.PPNet, model.construct_PPNet
    buf.seek(0)
    back = checkpoint.load_ppnet(buf)
    assert type(back) is model.PPNet and not hasattr(back, "precision")
    _same_module(ours, back)
    # without the shim: adopt() re-homes a PPNet-shaped module
    fake.PPNet = PPNet
    buf.seek(0)
    plain = torch.load(buf, weights_only=False)
    assert type(plain) is PPNet
    _same_module(ours, checkpoint.adopt(plain))


@pytest.mark.gpu
def test_loaded_checkpoint_runs_on_the_gpu(device, monkeypatch):
    """eval_valid.py:33-35: torch.load -> .cuda() -> forward; logits / distances equal the saved
    module's, i.e. the loaded object runs the HIP prototype layer. The backbone's convolutions run
    on torch's native path here: MIOpen may pick another solver for the second call (workspace-
    dependent), which changes the features' bits and says nothing about the checkpoint."""
    monkeypatch.setattr(torch.backends.cudnn, "enabled", False)
    checkpoint, _, _ = _pkg()
    ppnet = _ppnet((1, 1, 1, 1)).to(device).eval()
    img = torch.rand(2, 3, 129, 129, device=device)
    with torch.no_grad():
        logits, dist = ppnet(img)
    buf = io.BytesIO()
    checkpoint.save_ppnet(ppnet, buf)
    buf.seek(0)
    back = checkpoint.load_ppnet(buf).to(device).eval()
    with torch.no_grad():
        l2, d2 = back(img)
    torch.cuda.synchronize()
    assert torch.equal(logits, l2) and torch.equal(dist, d2)
    assert logits.shape == (2, 17, 17, 19) and dist.shape == (2, 190, 17, 17)
