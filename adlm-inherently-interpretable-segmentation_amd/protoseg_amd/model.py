"""PPNet with the reference's nn.Module surface, its prototype layer on the HIP kernels.

Mirrors reference model.py:39-418 (class ``PPNet`` and ``construct_PPNet``): same
constructor arguments, attributes, properties and methods, so segmentation/module.py,
segmentation/push.py and the eval scripts call it unchanged. What changes is underneath:
``_l2_convolution`` and ``forward_from_conv_features`` run one fused HIP kernel
(``protoseg_l2_fwd``) instead of 2 conv2d + 9 elementwise passes + Linear, and their
backward runs the two fused backward kernels (``protoseg_l2_bwd``).

There is no CPU path: calling the prototype layer on CPU tensors raises ProtosegError.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from ._lib import ProtosegError
from .deeplab import deeplabv2_resnet101_features
from .receptive_field import compute_proto_layer_rf_info_v2

base_architecture_to_features = {
    "deeplabv2_resnet101": deeplabv2_resnet101_features,
}


def _log(msg: str) -> None:
    print(msg)


class PPNet(nn.Module):
    def __init__(self, features, img_size, prototype_shape, proto_layer_rf_info, num_classes, init_weights=True,
                 prototype_activation_function="log", add_on_layers_type="bottleneck",
                 bottleneck_stride: Optional[int] = None, patch_classification: bool = False):
        super().__init__()
        self.img_size = img_size
        self.epsilon = 1e-4
        self.precision = None  # None: ops.DEFAULT_PRECISION ("bf16x3"); or "bf16x6" / "f32"
        self.bottleneck_stride = bottleneck_stride
        self.patch_classification = patch_classification
        self.prototype_vectors = nn.Parameter(torch.rand(prototype_shape), requires_grad=True)  # model.py:54
        self.prototype_activation_function = prototype_activation_function

        # model.py:66-73: one-hot class identity, equal prototypes per class
        n_protos = self.prototype_vectors.shape[0]
        if n_protos % num_classes != 0:
            raise AssertionError("num_prototypes must be divisible by num_classes")
        per_class = n_protos // num_classes
        identity = torch.zeros(n_protos, num_classes)
        for i in range(num_classes):
            identity[i * per_class:(i + 1) * per_class, i] = 1
        self.prototype_class_identity = identity
        self.num_prototypes_per_class = per_class
        self.proto_layer_rf_info = proto_layer_rf_info
        self.features = features

        in_ch = self._add_on_in_channels(features)
        depth = self.prototype_vectors.shape[1]
        if add_on_layers_type.startswith("bottleneck"):  # model.py:99-123
            layers = []
            if add_on_layers_type == "bottleneck_pool":
                layers += [nn.Conv2d(in_ch, in_ch, kernel_size=3, padding=1, stride=self.bottleneck_stride), nn.ReLU()]
            cur = in_ch
            while cur > depth or len(layers) == 0:
                out = max(depth, cur // 2)
                layers += [nn.Conv2d(cur, out, kernel_size=1), nn.ReLU(), nn.Conv2d(out, out, kernel_size=1)]
                if out > depth:
                    layers.append(nn.ReLU())
                else:
                    if out != depth:
                        raise AssertionError("bottleneck width mismatch")
                    layers.append(nn.Sigmoid())
                cur = cur // 2
            self.add_on_layers = nn.Sequential(*layers)
        elif add_on_layers_type == "deeplab_simple":  # model.py:124-128
            _log("deeplab_simple add_on_layers")
            self.add_on_layers = nn.Sequential(nn.Sigmoid())
        else:
            self.add_on_layers = nn.Sequential(
                nn.Conv2d(in_ch, depth, kernel_size=1), nn.ReLU(), nn.Conv2d(depth, depth, kernel_size=1), nn.Sigmoid())

        # model.py:140-141: kept for checkpoint / prune parity; the kernels never read it
        self.ones = nn.Parameter(torch.ones(self.prototype_vectors.shape), requires_grad=False)
        self.last_layer = nn.Linear(n_protos, num_classes, bias=False)
        if init_weights:
            self._initialize_weights()

    @staticmethod
    def _add_on_in_channels(features) -> int:
        """model.py:81-95: width of the last feature conv (the second-to-last for DeepLab/MSC)."""
        name = str(features).upper()
        if name.startswith("VGG") or name.startswith("RES"):
            return [m for m in features.modules() if isinstance(m, nn.Conv2d)][-1].out_channels
        if name.startswith("DENSE"):
            return [m for m in features.modules() if isinstance(m, nn.BatchNorm2d)][-1].num_features
        if name.startswith("DEEPLAB"):
            return [m for m in features.modules() if isinstance(m, nn.Conv2d)][-2].out_channels
        if name.startswith("MSC"):
            return [m for m in features.base.modules() if isinstance(m, nn.Conv2d)][-2].out_channels
        raise Exception(f"{name[:10]} base_architecture NOT implemented")

    # --- properties (model.py:149-159) -------------------------------------------------------
    @property
    def prototype_shape(self):
        return self.prototype_vectors.shape

    @property
    def num_prototypes(self):
        return self.prototype_vectors.shape[0]

    @property
    def num_classes(self):
        return self.prototype_class_identity.shape[1]

    # --- forward pieces ------------------------------------------------------------------------
    def run_last_layer(self, prototype_activations):
        return self.last_layer(prototype_activations)

    def conv_features(self, x):
        """model.py:164-175"""
        x = self.features(x)
        if isinstance(x, list):
            return [self.add_on_layers(x_scaled) for x_scaled in x]
        return self.add_on_layers(x)

    def _kernel_activation(self) -> Optional[str]:
        f = self.prototype_activation_function
        return f if isinstance(f, str) and f in ops.ACT_KINDS else None

    def _l2_convolution(self, x):
        """model.py:203-221 on the HIP kernel: relu(||x||^2 - 2 x.p + ||p||^2), [B, P, H, W]."""
        return ops.l2_distances(x, self.prototype_vectors, self.epsilon, getattr(self, "precision", None))

    def prototype_distances(self, x):
        return self._l2_convolution(self.conv_features(x))

    def distance_2_similarity(self, distances):
        """model.py:231-237 (elementwise; the fused kernel applies the same formula in-register)."""
        if self.prototype_activation_function == "log":
            return torch.log((distances + 1) / (distances + self.epsilon))
        if self.prototype_activation_function == "linear":
            return -distances
        return self.prototype_activation_function(distances)

    def _sigmoid_free_add_on(self):
        """The add-on layers minus their final nn.Sigmoid (model.py:124-128 and the bottleneck /
        regular add-ons all end in one) when forward() can hand the pre-activation to the layer
        kernels, which apply the sigmoid on load (sigmoid(X) never materialised); else None."""
        if not getattr(self, "fuse_add_on_sigmoid", True) or not getattr(self, "patch_classification", False):
            return None
        layers = list(self.add_on_layers)
        if not layers or not isinstance(layers[-1], nn.Sigmoid) or self._kernel_activation() is None:
            return None
        return nn.Sequential(*layers[:-1])

    def forward(self, x, **kwargs):
        head = self._sigmoid_free_add_on()
        if head is not None:  # conv_features() without its sigmoid, fused into the layer's load
            feats = self.features(x)
            if isinstance(feats, list):
                return [self.forward_from_conv_features(head(f), x_sigmoid=True, **kwargs) for f in feats]
            return self.forward_from_conv_features(head(feats), x_sigmoid=True, **kwargs)
        conv_features = self.conv_features(x)
        if isinstance(conv_features, list):
            return [self.forward_from_conv_features(c, **kwargs) for c in conv_features]
        return self.forward_from_conv_features(conv_features, **kwargs)

    def forward_with_features(self, x, **kwargs):
        conv_features = self.conv_features(x)
        if isinstance(conv_features, list):
            results = [self.forward_from_conv_features(c, **kwargs) for c in conv_features]
            return [(r[0], r[1], c) for r, c in zip(results, conv_features)]
        logits, distances = self.forward_from_conv_features(conv_features, **kwargs)
        return logits, distances, conv_features

    def forward_from_conv_features(self, conv_features, return_activations=False, return_distances=False,
                                   x_sigmoid=False):
        """model.py:259-299. Patch classification: one fused kernel gives distances (NCHW) and
        logits (NHWC) — the permute / activation / Linear / reshape of model.py:271-278 included.
        x_sigmoid=True: ``conv_features`` is the add-on's pre-activation (see forward())."""
        if isinstance(conv_features, list):
            return [self.forward_from_conv_features(c, x_sigmoid=x_sigmoid) for c in conv_features]
        act_name = self._kernel_activation()
        if x_sigmoid and not (getattr(self, "patch_classification", False) and act_name is not None):
            conv_features, x_sigmoid = torch.sigmoid(conv_features), False
        if getattr(self, "patch_classification", False):
            if act_name is None:  # a user-supplied activation: distances on the kernel, the rest in torch
                distances = self._l2_convolution(conv_features)
                b, p, h, w = distances.shape
                acts = self.distance_2_similarity(distances.permute(0, 2, 3, 1).reshape(-1, p))
                logits = self.run_last_layer(acts).reshape(b, h, w, -1)
                return (logits, acts) if return_activations else (logits, distances)
            distances, logits, acts = ops.prototype_layer(
                conv_features, self.prototype_vectors, self.last_layer.weight, self.epsilon, act_name,
                with_dist=not return_activations, with_logits=True, with_act=return_activations,
                precision=getattr(self, "precision", None), x_sigmoid=x_sigmoid)
            return (logits, acts) if return_activations else (logits, distances)

        # ProtoPNet global min pooling (model.py:284-299); distances from the kernel
        distances = self._l2_convolution(conv_features)
        min_distances = -F.max_pool2d(-distances, kernel_size=(distances.size()[2], distances.size()[3]))
        min_distances = min_distances.view(-1, self.num_prototypes)
        logits = self.run_last_layer(self.distance_2_similarity(min_distances))
        if return_distances:
            return logits, min_distances, distances
        return logits, min_distances

    def push_forward(self, x):
        """model.py:301-309"""
        conv_output = self.conv_features(x)
        if isinstance(conv_output, list):
            return [(c, self._l2_convolution(c)) for c in conv_output]
        return conv_output, self._l2_convolution(conv_output)

    # --- prototype bookkeeping -----------------------------------------------------------------
    def prune_prototypes(self, prototypes_to_prune):
        """model.py:311-336: drop prototypes, keeping the last layer / ones / identity aligned."""
        keep = sorted(set(range(self.num_prototypes)) - set(prototypes_to_prune))
        self.prototype_vectors = nn.Parameter(self.prototype_vectors.data[keep, ...], requires_grad=True)
        self.last_layer.in_features = self.num_prototypes
        self.last_layer.out_features = self.num_classes
        self.last_layer.weight.data = self.last_layer.weight.data[:, keep]
        self.ones = nn.Parameter(self.ones.data[keep, ...], requires_grad=False)
        self.prototype_class_identity = self.prototype_class_identity[keep, :]

    def __repr__(self):
        return ("PPNet(\n\tfeatures: {},\n\timg_size: {},\n\tprototype_shape: {},\n\tproto_layer_rf_info: {},\n"
                "\tnum_classes: {},\n\tepsilon: {}\n)").format(self.features, self.img_size, self.prototype_shape,
                                                              self.proto_layer_rf_info, self.num_classes,
                                                              self.epsilon)

    def set_last_layer_incorrect_connection(self, incorrect_strength):
        """model.py:359-371: 1 for the prototype's own class, ``incorrect_strength`` elsewhere."""
        positive = torch.t(self.prototype_class_identity)
        with torch.no_grad():
            self.last_layer.weight.copy_(1 * positive + incorrect_strength * (1 - positive))

    def _initialize_weights(self):
        for m in self.add_on_layers.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self.set_last_layer_incorrect_connection(incorrect_strength=-0.5)


def construct_PPNet(img_size=224, base_architecture="deeplabv2_resnet101", pretrained=True,
                    prototype_shape=(2000, 512, 1, 1), num_classes=200, prototype_activation_function="log",
                    add_on_layers_type="bottleneck", features: Optional[nn.Module] = None, **ppnet_kwargs):
    """model.py:389-418. ``features`` may be passed directly (e.g. a shallow backbone in tests);
    otherwise ``base_architecture`` selects the builder (DeepLabV2-ResNet101 here)."""
    if features is None:
        if base_architecture not in base_architecture_to_features:
            raise ProtosegError(f"backbone {base_architecture!r} is not part of this build "
                                f"(available: {sorted(base_architecture_to_features)})")
        features = base_architecture_to_features[base_architecture](pretrained=pretrained)
    if hasattr(features, "conv_info"):
        sizes, strides, paddings = features.conv_info()
    else:
        sizes, strides, paddings = [], [], []
    rf = compute_proto_layer_rf_info_v2(img_size=img_size, layer_filter_sizes=sizes, layer_strides=strides,
                                        layer_paddings=paddings, prototype_kernel_size=prototype_shape[2])
    return PPNet(features=features, img_size=img_size, prototype_shape=prototype_shape, proto_layer_rf_info=rf,
                 num_classes=num_classes, init_weights=True,
                 prototype_activation_function=prototype_activation_function,
                 add_on_layers_type=add_on_layers_type, **ppnet_kwargs)
