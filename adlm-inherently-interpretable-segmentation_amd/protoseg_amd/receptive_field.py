"""Receptive-field bookkeeping used at PPNet construction (receptive_field.py:4-33, 119-140).

Metadata only (push uses a stride grid, push.py:284-292); kept so ``proto_layer_rf_info``
has the reference's value.
"""
from __future__ import annotations

import math


def compute_layer_rf_info(layer_filter_size, layer_stride, layer_padding, previous_layer_rf_info):
    n_in, j_in, r_in, start_in = previous_layer_rf_info
    if layer_padding == "SAME":
        n_out = math.ceil(float(n_in) / float(layer_stride))
        rem = n_in % layer_stride
        pad = max(layer_filter_size - (layer_stride if rem == 0 else rem), 0)
    elif layer_padding == "VALID":
        n_out = math.ceil(float(n_in - layer_filter_size + 1) / float(layer_stride))
        pad = 0
    else:
        pad = layer_padding * 2
        n_out = math.floor((n_in - layer_filter_size + pad) / layer_stride) + 1
    p_left = math.floor(pad / 2)
    return [n_out, j_in * layer_stride, r_in + (layer_filter_size - 1) * j_in,
            start_in + ((layer_filter_size - 1) / 2 - p_left) * j_in]


def compute_proto_layer_rf_info_v2(img_size, layer_filter_sizes, layer_strides, layer_paddings,
                                   prototype_kernel_size):
    if not (len(layer_filter_sizes) == len(layer_strides) == len(layer_paddings)):
        raise ValueError("layer_filter_sizes, layer_strides and layer_paddings differ in length")
    rf_info = [img_size, 1, 1, 0.5]
    for f, s, p in zip(layer_filter_sizes, layer_strides, layer_paddings):
        rf_info = compute_layer_rf_info(f, s, p, rf_info)
    return compute_layer_rf_info(prototype_kernel_size, 1, "VALID", rf_info)
