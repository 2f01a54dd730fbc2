"""Checkpoints in the reference's format: whole-module pickles of ``PPNet``.

The reference saves the module object itself, not a state dict (segmentation/module.py:292, 297;
segmentation/train.py:192-193) and reloads it with a bare ``torch.load(path)`` (train.py:60, 64,
153, 195, 200; eval_valid.py:33; segmentation/run_pruning.py:27). What that means here:

* A checkpoint written by this build pickles ``protoseg_amd.model.PPNet`` (pickle records the
  class's defining module), so any process that can import ``protoseg_amd`` loads it.
* A checkpoint written by the reference pickles ``model.PPNet`` (plus its backbone classes). With
  INTEGRATION.md's shim (``from protoseg_amd.model import PPNet`` at the end of the reference's
  ``model.py``) that name resolves to this build's class, and pickle restores the reference's
  ``__dict__`` onto it: every attribute the reference's constructor sets (model.py:39-147) is one
  this class reads, and the ones it adds (``precision``, ``fuse_add_on_sigmoid``) default when
  absent.
* The state-dict keys are the reference's: ``prototype_vectors``, ``ones``, ``last_layer.weight``,
  ``features.base.*`` (DeepLabV2 names, deeplab_features.py:8-49), ``add_on_layers.*``; a reference
  state dict loads with ``strict=True`` (tests/test_checkpoint.py).

Since torch 2.6 a bare ``torch.load`` defaults to ``weights_only=True``, which refuses module
pickles, so the reference's own call no longer loads its own checkpoints on this stack.
``load_ppnet`` is that call with ``weights_only=False``: unpickling runs code from the file, so
use it only on checkpoints you wrote (the reference's trust model).
"""
from __future__ import annotations

from typing import Mapping, Optional

import torch
from torch import nn

from .model import PPNet


def save_ppnet(ppnet: nn.Module, f) -> None:
    """module.py:292 / train.py:192: ``torch.save(obj=ppnet, f=...)``."""
    torch.save(obj=ppnet, f=f)


def load_ppnet(f, map_location=None) -> nn.Module:
    """train.py:60 / eval_valid.py:33: ``torch.load(path)`` of a whole-module checkpoint (yours)."""
    obj = torch.load(f, map_location=map_location, weights_only=False)
    if not isinstance(obj, nn.Module):
        raise TypeError(f"{type(obj).__name__} is not a whole-module checkpoint; use load_state_dict_into")
    return obj


def load_state_dict_into(ppnet: PPNet, state_dict: Mapping[str, torch.Tensor], strict: bool = True):
    """Load a (reference-keyed) state dict; a pruned checkpoint's smaller P is adopted first
    (model.py:311-336 shrinks prototype_vectors, ones, the last layer's columns and the identity)."""
    p_new = state_dict.get("prototype_vectors")
    if p_new is not None and p_new.shape[0] != ppnet.num_prototypes:
        raise ValueError(f"checkpoint has {p_new.shape[0]} prototypes, model {ppnet.num_prototypes}: prune the "
                         "model first (PPNet.prune_prototypes) or load the whole-module checkpoint")
    return ppnet.load_state_dict(dict(state_dict), strict=strict)


def adopt(module: nn.Module, device: Optional[torch.device] = None) -> PPNet:
    """A PPNet-shaped module of another class (e.g. the reference's own, unpickled without the
    shim) as this build's ``PPNet``: same parameters and attributes, the prototype layer on HIP."""
    if isinstance(module, PPNet):
        return module if device is None else module.to(device)
    obj = PPNet.__new__(PPNet)
    obj.__dict__.update(module.__dict__)
    return obj if device is None else obj.to(device)
