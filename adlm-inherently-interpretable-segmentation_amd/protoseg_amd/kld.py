"""KLD similarity loss of segmentation/module.py:167-208 on the HIP kernels, with autograd.

The reference computes, per image and per class present in the (resized) label map, the
log_softmax of every prototype's distances over the class's pixels and the symmetric KL of
every prototype pair of the class, in a Python loop with host syncs; the loss is the mean
over all pairs of exp(-kld). ``kld_loss`` returns the same scalar from three kernels and
its backward produces d loss / d distances in one kernel, which then flows into the
prototype layer's backward as ``g_dist`` (protoseg_l2_bwd).

Reference quirks kept (oracle/kld_oracle.py): ``target_img`` holds raw label values with
0 = void and the prototype column for label value c is c itself, so void pixels pair with
class-0 prototypes and label value ``num_classes`` is skipped (module.py:170-178).
"""
from __future__ import annotations

import warnings
import weakref
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib

MAX_PER_CLASS = 32  # prototypes per class the kernels hold (kld.hip kKldMaxPerClass)

_LABEL_DTYPES = {torch.int64: _lib.I64, torch.int32: _lib.I32, torch.uint8: _lib.U8}


def _labels(target_img: Tensor, B: int) -> Tuple[Tensor, int]:
    t = target_img.reshape(B, -1)
    if t.dtype not in _LABEL_DTYPES:
        t = t.to(torch.int64)
    return t.contiguous(), _LABEL_DTYPES[t.dtype]


@torch.library.custom_op("protoseg::kld_forward", mutates_args=(), device_types="cuda")
def kld_forward(distances: Tensor, target_img: Tensor, proto_class: Tensor, num_classes: int,
                max_per_class: int) -> Tuple[Tensor, Tensor, Tensor]:
    """Returns (loss [] f32, n_pairs [] int32, workspace [bytes] uint8 for the backward)."""
    dev = _lib.require_device(distances, target_img, proto_class)
    d = distances.contiguous().float()
    B, P = d.shape[0], d.shape[1]
    HW = d[0, 0].numel()
    t, ldt = _labels(target_img, B)
    if t.shape[1] != HW:
        raise _lib.ProtosegError(f"target_img has {t.shape[1]} pixels per image, distances {HW}")
    pc = proto_class.to(torch.int32).contiguous()
    lib = _lib.load()
    ws = torch.empty(lib.protoseg_kld_workspace_size(B, P, HW, num_classes), device=dev, dtype=torch.uint8)
    loss = torch.empty((), device=dev, dtype=torch.float32)
    npairs = torch.empty((), device=dev, dtype=torch.int32)
    with torch.cuda.device(dev):
        _lib.call("protoseg_kld_forward", _lib.ptr(d), B, P, HW, _lib.ptr(t), ldt, _lib.ptr(pc), int(num_classes),
                  int(max_per_class), _lib.ptr(loss), _lib.ptr(npairs), _lib.ptr(ws), ws.numel(), _lib.stream_of(dev))
    return loss, npairs, ws


@kld_forward.register_fake
def _(distances, target_img, proto_class, num_classes, max_per_class):
    B, P = distances.shape[0], distances.shape[1]
    n = _lib.load().protoseg_kld_workspace_size(B, P, distances[0, 0].numel(), num_classes)
    return (distances.new_empty((), dtype=torch.float32), distances.new_empty((), dtype=torch.int32),
            distances.new_empty((n,), dtype=torch.uint8))


# protoseg_kld_backward_ex writes its per-pair coefficients into a buffer of its own
# (protoseg_kld_coef_bytes) and only reads the workspace, so the op mutates none of its inputs
# (mutates_args=() holds for torch.library.opcheck and functionalization) without copying the
# workspace. This is the dense fallback path (hooks, explicit-input passes, the wide
# family); the training path's compact backward computes its coefficients in LDS and writes nothing
# into the workspace.
@torch.library.custom_op("protoseg::kld_backward", mutates_args=(), device_types="cuda")
def kld_backward(distances: Tensor, target_img: Tensor, proto_class: Tensor, num_classes: int, max_per_class: int,
                 workspace: Tensor, g_loss: Tensor) -> Tensor:
    """d(g_loss * loss) / d distances, dense, shaped like ``distances``."""
    dev = _lib.require_device(distances, target_img, proto_class, workspace, g_loss)
    d = distances.contiguous().float()
    B, P = d.shape[0], d.shape[1]
    HW = d[0, 0].numel()
    t, ldt = _labels(target_img, B)
    pc = proto_class.to(torch.int32).contiguous()
    g = g_loss.to(torch.float32).contiguous()
    g_dist = torch.empty_like(d)
    coef = torch.empty(_lib.load().protoseg_kld_coef_bytes(B, int(num_classes)), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.call("protoseg_kld_backward_ex", _lib.ptr(d), B, P, HW, _lib.ptr(t), ldt, _lib.ptr(pc), int(num_classes),
                  int(max_per_class), _lib.ptr(g), _lib.ptr(workspace), workspace.numel(), _lib.ptr(coef),
                  coef.numel(), _lib.ptr(g_dist), _lib.stream_of(dev))
    return g_dist


@kld_backward.register_fake
def _(distances, target_img, proto_class, num_classes, max_per_class, workspace, g_loss):
    return torch.empty_like(distances, dtype=torch.float32)


def _setup_context(ctx, inputs, output):
    distances, target_img, proto_class, num_classes, max_per_class = inputs
    _, _, ws = output
    ctx.save_for_backward(distances, target_img, proto_class, ws)
    ctx.num_classes = num_classes
    ctx.max_per_class = max_per_class
    ctx.mark_non_differentiable(output[1], output[2])


def _backward(ctx, g_loss, g_npairs, g_ws):
    distances, target_img, proto_class, ws = ctx.saved_tensors
    if g_loss is None or not ctx.needs_input_grad[0]:
        return None, None, None, None, None
    g = kld_backward(distances, target_img, proto_class, ctx.num_classes, ctx.max_per_class, ws, g_loss)
    return g.to(distances.dtype), None, None, None, None


torch.library.register_autograd("protoseg::kld_forward", _backward, setup_context=_setup_context)


def kld_backward_compact(distances: Tensor, target_img: Tensor, proto_class: Tensor, num_classes: int,
                         max_per_class: int, workspace: Tensor, g_loss: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """The backward in its compact layout (protoseg_kld_backward_compact): (g_cls [B*HW, mpc] f32,
    pix_cls [B*HW] int32, proto_slot [P] int32); see include/protoseg_hip.h."""
    dev = _lib.require_device(distances, target_img, proto_class, workspace, g_loss)
    d = distances.contiguous().float()
    B, P = d.shape[0], d.shape[1]
    HW = d[0, 0].numel()
    t, ldt = _labels(target_img, B)
    pc = proto_class.to(torch.int32).contiguous()
    g = g_loss.to(torch.float32).contiguous()
    g_cls = torch.empty((B * HW, max_per_class), device=dev, dtype=torch.float32)
    pix_cls = torch.empty((B * HW,), device=dev, dtype=torch.int32)
    proto_slot = torch.empty((P,), device=dev, dtype=torch.int32)
    with torch.cuda.device(dev):
        _lib.call("protoseg_kld_backward_compact", _lib.ptr(d), B, P, HW, _lib.ptr(t), ldt, _lib.ptr(pc),
                  int(num_classes), int(max_per_class), _lib.ptr(g), _lib.ptr(workspace), workspace.numel(),
                  _lib.ptr(g_cls), _lib.ptr(pix_cls), _lib.ptr(proto_slot), _lib.stream_of(dev))
    return g_cls, pix_cls, proto_slot


# A private leaf that every _KldToLayer node takes as an input (and never sends a gradient to):
# its AccumulateGrad node is in each KLD graph. In a plain backward() the engine runs every node
# of the graph, so it reports that node as executing; when the pass has explicit inputs
# (autograd.grad, backward(inputs=...)) it runs only the nodes that lead to them, and the probe is
# never one of them. That tells the two kinds of pass apart from inside the backward.
_probe_state: dict = {}


def _graph_probe(device) -> Tuple[Tensor, object]:
    hit = _probe_state.get(str(device))
    if hit is None:
        probe = torch.zeros((), device=device, requires_grad=True)
        node = torch.autograd.graph.get_gradient_edge(probe).node  # its AccumulateGrad
        hit = _probe_state[str(device)] = (probe, node)
    return hit


def _pass_runs_every_node(probe_node) -> bool:
    """True in a backward pass without explicit inputs (every node of the graph executes)."""
    try:
        return bool(torch._C._will_engine_execute_node(probe_node))
    except (AttributeError, RuntimeError):  # no engine introspection: treat as explicit inputs
        _warn_no_introspection()
        return False


def _layer_backward_runs(layer_node) -> bool:
    """Whether the current backward pass will run the prototype layer's backward past its own
    node, i.e. consume a deposit: some node behind it (x's producer, the prototypes' or the last
    layer's AccumulateGrad) executes."""
    if layer_node is None:
        return False
    try:
        return any(torch._C._will_engine_execute_node(n) for n, _ in layer_node.next_functions if n is not None)
    except (AttributeError, RuntimeError):  # no engine introspection: always the dense gradient
        _warn_no_introspection()
        return False


_warned_introspection = False


def _warn_no_introspection():
    """Once per process: this torch has no autograd-engine introspection, so every KLD backward
    takes the dense [B, P, H, W] gradient instead of the compact hand-off (slower, same values)."""
    global _warned_introspection
    if not _warned_introspection:
        _warned_introspection = True
        warnings.warn("protoseg KLD: torch._C._will_engine_execute_node is unavailable; the KLD gradient takes "
                      "the dense path", RuntimeWarning, stacklevel=3)


class _KldToLayer(torch.autograd.Function):
    """kld_forward whose backward hands the compact gradient to the prototype layer that produced
    ``distances`` (ops.DistGradSink) instead of returning a dense [B, P, H, W] tensor.

    The hand-off is taken only in a plain ``backward()`` (no explicit inputs) that runs the
    layer's backward, with nothing observing the gradient at ``distances`` itself (``retain_grad``
    or a tensor hook). Any pass with explicit inputs (``autograd.grad``, ``backward(inputs=...)``)
    gets the dense gradient: ``distances`` may be one of its capture targets, and the engine does
    not say which tensors those are. So captures, hooks and ``retain_grad`` see the real values.
    Deposits carry the backward pass's graph-task id and the layer takes only its own pass's, so a
    ``retain_graph`` replay never sums a stale deposit."""

    @staticmethod
    def forward(ctx, distances, target_img, proto_class, num_classes, max_per_class, sink, layer_node, probe,
                probe_node):
        loss, npairs, ws = torch.ops.protoseg.kld_forward(distances, target_img, proto_class, num_classes,
                                                          max_per_class)
        ctx.save_for_backward(distances, target_img, proto_class, ws)
        ctx.num_classes, ctx.max_per_class, ctx.sink = num_classes, max_per_class, sink
        ctx.layer_node = layer_node
        ctx.probe_node = probe_node
        ctx.dist_ref = sink.dist_ref
        ctx.mark_non_differentiable(npairs)
        return loss, npairs

    @staticmethod
    def backward(ctx, g_loss, g_npairs):
        distances, target_img, proto_class, ws = ctx.saved_tensors
        none = (None,) * 8
        if g_loss is None or not ctx.needs_input_grad[0]:
            return (None,) + none
        d = ctx.dist_ref() if ctx.dist_ref is not None else None
        observed = d is not None and (d.retains_grad or bool(getattr(d, "_backward_hooks", None)))
        if observed or not _pass_runs_every_node(ctx.probe_node) or not _layer_backward_runs(ctx.layer_node):
            g = kld_backward(distances, target_img, proto_class, ctx.num_classes, ctx.max_per_class, ws, g_loss)
            return (g.to(distances.dtype),) + none
        g_cls, pix_cls, proto_slot = kld_backward_compact(distances, target_img, proto_class, ctx.num_classes,
                                                          ctx.max_per_class, ws, g_loss)
        return (ctx.sink.deposit(g_cls, pix_cls, proto_slot, ctx.max_per_class, distances),) + none


def kld_with_pairs(distances: Tensor, target_img: Tensor, proto_class: Tensor, num_classes: int,
                   max_per_class: int) -> Tuple[Tensor, Tensor]:
    """(loss, n_pairs) of module.py:167-208. When ``distances`` is the distances output of the
    HIP prototype layer and its backward can take the compact gradient, the gradient goes to the
    layer in that form (no [B, P, H, W] tensor); otherwise autograd gets the dense one."""
    sink = getattr(distances, "_protoseg_sink", None)
    if sink is not None and distances.requires_grad and torch.is_grad_enabled() and sink.accepts(max_per_class):
        probe, probe_node = _graph_probe(distances.device)
        return _KldToLayer.apply(distances, target_img, proto_class, int(num_classes), int(max_per_class), sink,
                                 distances.grad_fn, probe, probe_node)
    loss, npairs, _ = torch.ops.protoseg.kld_forward(distances, target_img, proto_class, int(num_classes),
                                                     int(max_per_class))
    return loss, npairs

_class_cache: dict = {}


def prototype_columns(prototype_class_identity: Tensor, device) -> Tuple[Tensor, int]:
    """(class column of each prototype as int32 on ``device``, max prototypes per class).

    module.py:173 selects the prototypes of class c as nonzero(identity[:, c]); with the
    reference's one-hot identity (model.py:66-71) that is argmax(identity[p]) == c. Cached per
    identity tensor version, so a training loop pays the host reduction once."""
    ident = prototype_class_identity
    key = (id(ident), ident._version, ident.data_ptr(), tuple(ident.shape), str(device))
    hit = _class_cache.get(key)
    # the entry holds a weak reference to its tensor: a new tensor that reuses a freed one's id
    # and storage address is a miss, not the freed tensor's columns
    if hit is not None and hit[0]() is ident:
        return hit[1]
    host = ident.detach().to("cpu")
    if host.dim() != 2 or not bool(((host != 0).sum(1) == 1).all()):
        raise _lib.ProtosegError("prototype_class_identity must be one-hot per prototype (model.py:66-71)")
    counts = (host != 0).sum(0)
    mpc = max(1, int(counts.max()))
    if mpc > MAX_PER_CLASS:
        raise _lib.ProtosegError(f"{mpc} prototypes in one class; the KLD kernels hold at most {MAX_PER_CLASS}")
    cols = host.abs().argmax(1).to(torch.int32).to(device)
    if len(_class_cache) > 16:
        _class_cache.clear()
    _class_cache[key] = (weakref.ref(ident), (cols, mpc))
    return cols, mpc


def kld_loss(distances: Tensor, target_img: Tensor, prototype_class_identity: Tensor,
             max_per_class: Optional[int] = None) -> Tensor:
    """module.py:167-208: mean over (image, class, prototype pair) of exp(-symmetric KL) of the
    per-prototype log_softmax of the distances over the class's pixels. 0-dim f32 tensor
    (0 when no pair exists), differentiable with respect to ``distances``.

    distances [B, P, h, w] (PPNet.forward's second output); target_img [B, h*w] or [B, h, w]
    label values (0 = void); prototype_class_identity [P, K] one-hot."""
    cols, mpc = prototype_columns(prototype_class_identity, distances.device)
    if max_per_class is not None:
        mpc = int(max_per_class)
    loss, _ = kld_with_pairs(distances, target_img, cols, int(prototype_class_identity.shape[1]), mpc)
    return loss
