"""torch.library custom ops over the C ABI: the prototype layer forward and its backward.

``prototype_layer(x, protos, w_last, ...)`` is the autograd-aware entry used by ``PPNet``:
one fused HIP kernel produces distances (NCHW), logits (NHWC) and optionally activations;
the backward recomputes distances from ``x`` and calls the two backward kernels.

Reference: model.py:203-221 (_l2_convolution), 231-237 (distance_2_similarity),
259-283 (forward_from_conv_features, patch_classification branch); the backward is the
autograd graph of those ops (the reference has no custom backward).
"""
from __future__ import annotations

import os
import weakref
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib

ACT_KINDS = {"log": _lib.ACT_LOG, "linear": _lib.ACT_LINEAR}
PRECISIONS = _lib.PRECISIONS
# bf16x3: bf16 MFMA on 2-term split operands (|rel err| ~1e-5 on distances, the default);
# bf16x6: 3-term split (f32-class); f32: v_mfma_f32_32x32x2_f32 (exact f32 fma chain).
DEFAULT_PRECISION = os.environ.get("PROTOSEG_PRECISION", "bf16x3")


def precision_code(precision: Optional[str]) -> int:
    name = DEFAULT_PRECISION if precision is None else precision
    if name not in PRECISIONS:
        raise _lib.ProtosegError(f"precision {name!r} unknown (one of {sorted(PRECISIONS)})")
    return PRECISIONS[name]


def _x_dtype(x: Tensor) -> int:
    if x.dtype == torch.float32:
        return _lib.F32
    if x.dtype == torch.bfloat16:
        return _lib.BF16
    if x.dtype == torch.float16:
        return _lib.F16
    raise _lib.ProtosegError(f"feature map dtype {x.dtype} unsupported (float32, bfloat16 or float16)")


def supported(C: int, P: int, K: int) -> bool:
    return bool(_lib.load().protoseg_l2_supported(C, P, K))


def x_dtype_supported(C: int, P: int, K: int, dtype: torch.dtype) -> bool:
    """Whether the kernels read feature maps of `dtype` natively for (C, P, K)
    (protoseg_l2_x_dtype_supported: fp16 in the wide family); else the layer widens to f32."""
    code = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float16: _lib.F16}.get(dtype)
    return code is not None and bool(_lib.load().protoseg_l2_x_dtype_supported(C, P, K, code))


def bwd_reads_dist(C: int, P: int, K: int, precision: int) -> bool:
    """Whether the backward at this shape reads the forward's distances instead of recomputing
    them (protoseg_l2_bwd_reads_dist: the wide family)."""
    return bool(_lib.load().protoseg_l2_bwd_reads_dist(C, P, K, int(precision)))


def x_sigmoid_supported(x: Tensor, P: int, K: int, precision: Optional[str] = None) -> bool:
    """Whether the kernels can apply the add-on's sigmoid on load for this call."""
    B, C, H, W = x.shape
    return bool(_lib.load().protoseg_l2_x_sigmoid_supported(B, C, H, W, P, K, precision_code(precision)))


def max_protos(C: int, precision: Optional[str] = None) -> int:
    """Largest P one layer call serves at (C, precision) (protoseg_l2_max_protos)."""
    return int(_lib.load().protoseg_l2_max_protos(C, precision_code(precision)))


def train_operands_bytes(C: int, P: int, K: int, precision: int) -> int:
    """Bytes of the backward's operand images the forward can build (protoseg_l2_train_operands_bytes);
    0 when the backward at this shape / precision would not read them."""
    return int(_lib.load().protoseg_l2_train_operands_bytes(C, P, K, int(precision)))


@torch.library.custom_op("protoseg::l2_forward", mutates_args=(), device_types="cuda")
def l2_forward(x: Tensor, protos: Tensor, w_last: Tensor, eps: float, act_kind: int, precision: int,
               with_dist: bool, with_logits: bool, with_act: bool,
               with_operands: bool = False) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Fused prototype-layer forward. Returns (dist [B,P,H,W], logits [B,H,W,K], act [B*H*W,P],
    operands): outputs not requested are empty tensors. with_operands: the training backward's
    operand images (uint8, protoseg_l2_fwd_ex) built in the forward's prep launch, for
    l2_backward(..., operands=...); empty when the backward at this shape would not read them."""
    dev = _lib.require_device(x, protos, w_last)
    x = x.contiguous()
    protos = protos.contiguous()
    w_last = w_last.contiguous()
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    f32 = dict(device=dev, dtype=torch.float32)
    dist = torch.empty((B, P, H, W) if with_dist else (0,), **f32)
    logits = torch.empty((B, H, W, K) if with_logits else (0,), **f32)
    act = torch.empty((B * H * W, P) if with_act else (0,), **f32)
    nops = train_operands_bytes(C, P, K, precision) if with_operands else 0
    ops_buf = torch.empty(nops, device=dev, dtype=torch.uint8)
    with torch.cuda.device(dev):
        _lib.call("protoseg_l2_fwd_ex", _lib.ptr(x), _x_dtype(x), B, C, H, W, _lib.ptr(protos), P,
                  _lib.ptr(w_last), K, float(eps), int(act_kind), int(precision), _lib.ptr(dist), _lib.ptr(act),
                  _lib.ptr(logits), _lib.ptr(ops_buf) if nops else None, nops, _lib.stream_of(dev))
    return dist, logits, act, ops_buf


@l2_forward.register_fake
def _(x, protos, w_last, eps, act_kind, precision, with_dist, with_logits, with_act, with_operands=False):
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    e = lambda *s: x.new_empty(s, dtype=torch.float32)  # noqa: E731
    nops = train_operands_bytes(C, P, K, precision) if with_operands else 0
    return (e(B, P, H, W) if with_dist else e(0), e(B, H, W, K) if with_logits else e(0),
            e(B * H * W, P) if with_act else e(0), x.new_empty(nops, dtype=torch.uint8))


def _operands_args(operands: Optional[Tensor]):
    """(pointer, bytes) of an operands buffer for the _ex calls; (None, 0) without one."""
    if operands is None or operands.numel() == 0:
        return None, 0
    return _lib.ptr(operands), operands.numel()


@torch.library.custom_op("protoseg::l2_backward", mutates_args=(), device_types="cuda")
def l2_backward(x: Tensor, protos: Tensor, w_last: Tensor, g_logits: Optional[Tensor], g_dist: Optional[Tensor],
                eps: float, act_kind: int, precision: int, need_x: bool, need_protos: bool,
                need_w: bool, operands: Optional[Tensor] = None,
                dist: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """Backward of l2_forward with respect to (x, protos, w_last); unrequested grads are empty.
    With X_SIGMOID in act_kind, g_x is the gradient w.r.t. the pre-activation. operands: the
    forward's with_operands output (same protos / w_last values), read instead of a prep launch.
    dist: the forward's distances, read instead of recomputed where bwd_reads_dist (the wide
    family: protoseg_l2_bwd_saved); same gradients bit for bit."""
    dev = _lib.require_device(x, protos, w_last, g_logits, g_dist)
    x = x.contiguous()
    protos = protos.contiguous()
    w_last = w_last.contiguous()
    g_logits = g_logits.contiguous().float() if g_logits is not None else None
    g_dist = g_dist.contiguous().float() if g_dist is not None else None
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    need_w = need_w and g_logits is not None
    g_x = torch.empty_like(x) if need_x else x.new_empty(0)
    g_p = torch.empty((P, C), device=dev, dtype=torch.float32) if need_protos else x.new_empty(0, dtype=torch.float32)
    g_w = torch.empty((K, P), device=dev, dtype=torch.float32) if need_w else x.new_empty(0, dtype=torch.float32)
    if need_w is False and g_logits is None and need_protos is False and need_x is False:
        return g_x, g_p, g_w
    lib = _lib.load()
    ops_ptr, ops_bytes = _operands_args(operands)
    with torch.cuda.device(dev):
        # slabs of g_P / g_W, every X_SIGMOID backward, and the wide family's D / G_s buffers (any
        # request, g_x alone included): the size query is host-only but depends on the device's
        # CU count (one slab per workgroup), so it runs inside the device context; torch's
        # allocator caches the block
        ws_bytes = lib.protoseg_l2_bwd_workspace_size(B, C, H, W, P, K)
        ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8) if ws_bytes else None
        if dist is not None and dist.numel():
            _lib.call("protoseg_l2_bwd_saved", _lib.ptr(x), _x_dtype(x), B, C, H, W, _lib.ptr(protos), P,
                      _lib.ptr(w_last), K, float(eps), int(act_kind), int(precision), _lib.ptr(dist.contiguous()),
                      _lib.ptr(g_logits), _lib.ptr(g_dist), _lib.ptr(g_x), _lib.ptr(g_p), _lib.ptr(g_w),
                      _lib.ptr(ws), ws_bytes, _lib.stream_of(dev))
        else:
            _lib.call("protoseg_l2_bwd_ex", _lib.ptr(x), _x_dtype(x), B, C, H, W, _lib.ptr(protos), P,
                      _lib.ptr(w_last), K, float(eps), int(act_kind), int(precision), _lib.ptr(g_logits),
                      _lib.ptr(g_dist), _lib.ptr(g_x), _lib.ptr(g_p), _lib.ptr(g_w), _lib.ptr(ws), ws_bytes, ops_ptr,
                      ops_bytes, _lib.stream_of(dev))
    return g_x, g_p, g_w


@l2_backward.register_fake
def _(x, protos, w_last, g_logits, g_dist, eps, act_kind, precision, need_x, need_protos, need_w, operands=None,
      dist=None):
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    need_w = need_w and g_logits is not None
    return (torch.empty_like(x) if need_x else x.new_empty(0),
            x.new_empty((P, C), dtype=torch.float32) if need_protos else x.new_empty(0, dtype=torch.float32),
            x.new_empty((K, P), dtype=torch.float32) if need_w else x.new_empty(0, dtype=torch.float32))


class DistGradSink:
    """Hand-off of the KLD loss's distance gradient to this layer's backward in its compact layout.

    The KLD gradient (module.py:167-208) is non-zero only at the prototypes of each pixel's own
    class, so a dense [B, P, H, W] tensor is mostly zeros written and read back. ``l2_forward``
    attaches one sink to its distances output; ``kld.kld_loss`` on those distances deposits the
    compact (g_cls, pix_cls, proto_slot, max_per_class) triple here and returns an expanded zero
    to autograd, and this layer's backward hands the deposit to ``protoseg_l2_bwd_kld``, which
    expands it in registers. Gradients from any other consumer of the distances still arrive
    densely through autograd and are added. If the layer backward cannot take the compact form
    (a shape / precision the kernels do not serve, a gradient through the activations), the
    deposits are expanded with ``protoseg_kld_expand`` first: same values either way."""

    __slots__ = ("shape", "compact_ok", "deposits", "zero", "dist_ref")

    def __init__(self, shape, compact_ok: bool):
        self.shape = shape          # (B, C, H, W, P, K, x_dtype, precision)
        self.compact_ok = compact_ok
        self.deposits = []          # (graph task id, (g_cls, pix_cls, proto_slot, max_per_class))
        self.zero = None
        self.dist_ref = None        # weak reference to the distances tensor (retain_grad / hook checks)

    def accepts(self, max_per_class: int) -> bool:
        """Whether a KLD backward on these distances should deposit its compact form."""
        if not self.compact_ok:
            return False
        return bool(_lib.load().protoseg_l2_bwd_kld_supported(*self.shape, int(max_per_class)))

    def deposit(self, g_cls: Tensor, pix_cls: Tensor, proto_slot: Tensor, max_per_class: int, like: Tensor) -> Tensor:
        self.deposits.append((_graph_task(), (g_cls, pix_cls, proto_slot, int(max_per_class))))
        if self.zero is None or self.zero.device != like.device:
            self.zero = torch.zeros((), device=like.device, dtype=like.dtype).expand(like.shape)
        return self.zero

    def is_zero(self, g: Optional[Tensor]) -> bool:
        z = self.zero
        return (g is not None and z is not None and g.shape == z.shape and g.stride() == z.stride()
                and g.data_ptr() == z.data_ptr())

    def take(self):
        """This backward pass's deposits (older passes' stale ones, e.g. of a pass that stopped at
        the distances, are dropped)."""
        task = _graph_task()
        d, self.deposits = self.deposits, []
        return [dep for t, dep in d if t == task]


def _graph_task() -> int:
    try:
        return int(torch._C._current_graph_task_id())
    except (AttributeError, RuntimeError):
        return -1


def expand_compact(deposit, B: int, P: int, HW: int, out: Optional[Tensor] = None) -> Tensor:
    """Dense [B, P, HW] g_dist of a compact KLD deposit (protoseg_kld_expand); added to ``out``."""
    g_cls, pix_cls, proto_slot, mpc = deposit
    dev = g_cls.device
    acc = out is not None
    if out is None:
        out = torch.empty((B, P, HW), device=dev, dtype=torch.float32)
    with torch.cuda.device(dev):
        _lib.call("protoseg_kld_expand", _lib.ptr(g_cls), _lib.ptr(pix_cls), _lib.ptr(proto_slot), B, P, HW, mpc,
                  1 if acc else 0, _lib.ptr(out), _lib.stream_of(dev))
    return out


@torch.library.custom_op("protoseg::l2_backward_kld", mutates_args=(), device_types="cuda")
def l2_backward_kld(x: Tensor, protos: Tensor, w_last: Tensor, g_logits: Optional[Tensor], g_cls: Tensor,
                    pix_cls: Tensor, proto_slot: Tensor, max_per_class: int, eps: float, act_kind: int, precision: int,
                    need_x: bool, need_protos: bool, need_w: bool,
                    operands: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """l2_backward with the KLD loss's compact distance gradient (protoseg_l2_bwd_kld): the
    kernels expand g_dist in registers instead of reading a dense [B, P, H, W] tensor."""
    dev = _lib.require_device(x, protos, w_last, g_logits, g_cls, pix_cls, proto_slot)
    x = x.contiguous()
    protos = protos.contiguous()
    w_last = w_last.contiguous()
    g_logits = g_logits.contiguous().float() if g_logits is not None else None
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    need_w = need_w and g_logits is not None
    g_x = torch.empty_like(x) if need_x else x.new_empty(0)
    g_p = torch.empty((P, C), device=dev, dtype=torch.float32) if need_protos else x.new_empty(0, dtype=torch.float32)
    g_w = torch.empty((K, P), device=dev, dtype=torch.float32) if need_w else x.new_empty(0, dtype=torch.float32)
    lib = _lib.load()
    ops_ptr, ops_bytes = _operands_args(operands)
    with torch.cuda.device(dev):
        ws_bytes = lib.protoseg_l2_bwd_workspace_size(B, C, H, W, P, K)  # (per device: see l2_backward)
        ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
        _lib.call("protoseg_l2_bwd_kld_ex", _lib.ptr(x), _x_dtype(x), B, C, H, W, _lib.ptr(protos), P,
                  _lib.ptr(w_last), K, float(eps), int(act_kind), int(precision), _lib.ptr(g_logits),
                  _lib.ptr(g_cls), _lib.ptr(pix_cls), _lib.ptr(proto_slot), int(max_per_class), _lib.ptr(g_x),
                  _lib.ptr(g_p), _lib.ptr(g_w), _lib.ptr(ws), ws_bytes, ops_ptr, ops_bytes, _lib.stream_of(dev))
    return g_x, g_p, g_w


@l2_backward_kld.register_fake
def _(x, protos, w_last, g_logits, g_cls, pix_cls, proto_slot, max_per_class, eps, act_kind, precision, need_x,
      need_protos, need_w, operands=None):
    B, C, H, W = x.shape
    P, K = protos.shape[0], w_last.shape[0]
    need_w = need_w and g_logits is not None
    return (torch.empty_like(x) if need_x else x.new_empty(0),
            x.new_empty((P, C), dtype=torch.float32) if need_protos else x.new_empty(0, dtype=torch.float32),
            x.new_empty((K, P), dtype=torch.float32) if need_w else x.new_empty(0, dtype=torch.float32))


def _setup_context(ctx, inputs, output):
    x, protos, w_last, eps, act_kind, precision, with_dist, with_logits, with_act = inputs[:9]
    # the forward-built operand images are saved like the inputs, so saved-tensor hooks see them
    # and the version check guards them (an empty tensor when the forward built none); so are the
    # distances where the backward reads them instead of recomputing (the wide family)
    dist_saved = output[0] if (with_dist and output[0].numel() and x.is_cuda and
                               bwd_reads_dist(x.shape[1], protos.shape[0], w_last.shape[0], precision)) else None
    ctx.save_for_backward(x, protos, w_last, output[3], dist_saved)
    ctx.eps = eps
    ctx.act_kind = act_kind
    ctx.precision = precision
    ctx.set_materialize_grads(False)  # unused outputs give None, not a zero-filled [B,P,H,W]
    ctx.sink = None
    dist = output[0]
    if with_dist and dist.numel() and x.is_cuda:
        B, C, H, W = x.shape
        trains = x.requires_grad and (protos.requires_grad or w_last.requires_grad)
        ctx.sink = DistGradSink((B, C, H, W, protos.shape[0], w_last.shape[0], _x_dtype(x), int(precision)), trains)
        ctx.sink.dist_ref = weakref.ref(dist)
        dist._protoseg_sink = ctx.sink


def _act_grad_as_dist_grad(x, protos, w_last, g_act, eps, act_kind, precision):
    """Gradient arriving at the activations (return_activations=True, model.py:280-281) as a
    distance gradient: g_d = g_act * d act / d d, with act = log((d+1)/(d+eps)) (model.py:233):
    1/(d+1) - 1/(d+eps) = (eps-1)/((d+1)(d+eps)); linear: -1. The distances are recomputed on the
    GPU by the forward kernel; the relu mask is applied by the backward kernel as for g_dist."""
    B, _, H, W = x.shape
    P = protos.shape[0]
    ga = g_act.reshape(B, H, W, P).permute(0, 3, 1, 2).float()
    if act_kind & ~_lib.X_SIGMOID == _lib.ACT_LINEAR:
        return -ga
    d = l2_forward(x, protos, w_last, eps, act_kind, precision, True, False, False)[0]
    return ga * ((eps - 1.0) / ((d + 1.0) * (d + eps)))


def _backward(ctx, g_dist, g_logits, g_act, g_operands=None):
    x, protos, w_last, operands, dist_saved = ctx.saved_tensors
    need_x, need_p, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
    sink = ctx.sink
    compact = sink.take() if sink is not None else []
    if sink is not None and sink.is_zero(g_dist):
        g_dist = None  # only the KLD loss consumed the distances: its gradient is in `compact`
    if g_act is not None:
        extra = _act_grad_as_dist_grad(x, protos, w_last, g_act, ctx.eps, ctx.act_kind, ctx.precision)
        g_dist = extra if g_dist is None else g_dist + extra
    B, _, H, W = x.shape
    P = protos.shape[0]
    if compact and (g_dist is not None or len(compact) > 1 or not (need_x and (need_p or need_w))):
        dense = g_dist.reshape(B, P, H * W).float().contiguous() if g_dist is not None else None
        for dep in compact:
            dense = expand_compact(dep, B, P, H * W, dense)
        g_dist, compact = dense.reshape(B, P, H, W), []
    if g_dist is None and g_logits is None and not compact:
        return None, None, None, None, None, None, None, None, None, None
    ops_buf = operands if operands.numel() else None
    if compact:
        g_cls, pix_cls, proto_slot, mpc = compact[0]
        g_x, g_p, g_w = l2_backward_kld(x, protos, w_last, g_logits, g_cls, pix_cls, proto_slot, mpc, ctx.eps,
                                        ctx.act_kind, ctx.precision, need_x, need_p, need_w and g_logits is not None,
                                        ops_buf)
    else:
        g_x, g_p, g_w = l2_backward(x, protos, w_last, g_logits, g_dist, ctx.eps, ctx.act_kind, ctx.precision, need_x,
                                    need_p, need_w and g_logits is not None, ops_buf, dist_saved)
    return (g_x if need_x else None, g_p if need_p else None, g_w if (need_w and g_w.numel()) else None,
            None, None, None, None, None, None, None)


torch.library.register_autograd("protoseg::l2_forward", _backward, setup_context=_setup_context)


def prototype_layer(x: Tensor, prototype_vectors: Tensor, last_layer_weight: Tensor, eps: float = 1e-4,
                    activation: str = "log", with_dist: bool = True, with_logits: bool = True,
                    with_act: bool = False, precision: Optional[str] = None,
                    x_sigmoid: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """Distances, logits and activations of the PPNet prototype layer.

    x: [B, C, H, W] add-on-layer output (float32, bfloat16 or float16: read natively where
    x_dtype_supported, else widened to f32); prototype_vectors: [P, C, kh, kw]
    or [P, C]; last_layer_weight: [K, P]. Returns (distances [B,P,H',W'], logits [B,H',W',K],
    activations [B*H'*W', P]) with unrequested outputs empty; H' = H - kh + 1, W' = W - kw + 1
    (k x k prototypes run on the unfolded map, C k k deep).

    x_sigmoid=True: x is the add-on layers' pre-activation and the layer input is sigmoid(x)
    (model.py:124-128's final nn.Sigmoid). The kernels apply it on load where
    protoseg_l2_x_sigmoid_supported says so (bf16x3, C = 64), so sigmoid(x) is never written to
    HBM and autograd returns the pre-activation's gradient; other shapes / precisions take
    torch.sigmoid first.
    """
    if activation not in ACT_KINDS:
        raise _lib.ProtosegError(f"activation {activation!r} has no HIP kernel ('log' or 'linear')")
    protos = prototype_vectors.reshape(prototype_vectors.shape[0], -1)
    kernel = tuple(prototype_vectors.shape[2:]) if prototype_vectors.dim() == 4 else (1, 1)
    if kernel != (1, 1):
        # k x k prototypes (model.py:203-221 is a general F.conv2d, no padding): the k x k
        # windows as columns (unfold, in prototype_vectors.reshape(P, -1)'s (c, dy, dx) order),
        # then the same kernels on 1x1 prototypes of depth C k k; autograd folds g_x back
        if prototype_vectors.shape[1] != x.shape[1]:
            raise _lib.ProtosegError(f"prototype depth {prototype_vectors.shape[1]} != feature channels {x.shape[1]}")
        B, C, H, W = x.shape
        kh, kw = kernel
        if kh > H or kw > W:
            raise _lib.ProtosegError(f"{kh}x{kw} prototypes on a {H}x{W} map")
        if x.dtype == torch.float16:
            x = x.float()
        if x_sigmoid:
            x, x_sigmoid = torch.sigmoid(x), False
        x = torch.nn.functional.unfold(x, (kh, kw)).reshape(B, C * kh * kw, H - kh + 1, W - kw + 1)
    if protos.shape[1] != x.shape[1]:
        raise _lib.ProtosegError(f"prototype depth {protos.shape[1]} != feature channels {x.shape[1]}")
    if x.dtype == torch.float16 and (x_sigmoid or not x_dtype_supported(x.shape[1], protos.shape[0],
                                                                         last_layer_weight.shape[0], torch.float16)):
        # fp16 feature maps (BASELINE config 5, DenseNet-161 fp16) outside the wide family: widened
        # exactly to f32 at the boundary; autograd narrows g_x back to fp16. The wide family reads
        # fp16 in its GEMM stages (no widening pass) and writes g_x as fp16.
        x = x.float()
    act_kind = ACT_KINDS[activation]
    if x_sigmoid:
        if x.is_cuda and x_sigmoid_supported(x, protos.shape[0], last_layer_weight.shape[0], precision):
            act_kind |= _lib.X_SIGMOID
        else:
            x = torch.sigmoid(x)
    prec = precision_code(precision)
    # a training forward builds the backward's operand images in its own prep launch (one prep
    # per step; the saved-tensor version check keeps them tied to these protos / weights)
    trains = (torch.is_grad_enabled() and x.is_cuda and x.requires_grad
              and (protos.requires_grad or last_layer_weight.requires_grad))
    return torch.ops.protoseg.l2_forward(x, protos, last_layer_weight, float(eps), act_kind, prec, with_dist,
                                         with_logits, with_act, trains)[:3]


def l2_distances(x: Tensor, prototype_vectors: Tensor, eps: float = 1e-4, precision: Optional[str] = None) -> Tensor:
    """model.py:203-221 _l2_convolution: squared L2 distance map [B, P, H, W]."""
    w_dummy = x.new_zeros((1, prototype_vectors.shape[0]), dtype=torch.float32)
    return prototype_layer(x, prototype_vectors, w_dummy, eps, "log", True, False, False, precision)[0]
