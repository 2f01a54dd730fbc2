#!/usr/bin/env python3
"""bench.py — ProtoSeg hot path on MI355X: prototype-layer training step + prototype push.

Workload (BASELINE.json metric: 513x513, 19 prototypes/class; configs[1] cityscapes_no_kld_imnet
otherwise): 513x513 crops -> 65x65 feature maps, C=64, P=361 (19 classes x 19), K=19; the
P=190 (10/class, the gin files' count) step is a side line with its own roofline. One "step" = the
prototype layer's forward (distances + logits, one fused kernel), backward (g_x, g_prototypes,
g_last_layer; one fused kernel per prototype chunk), the data-parallel gradient exchange when
N>1 (protoseg_amd.distributed.GradientBuckets: bucketed RCCL all-reduce, the exchange of
train.PatchClassificationStep) and the Adam update of P and W (module.py:391), over a batch of B
images per GPU.
Synthetic data (seed 20220227): X = sigmoid(N(0, 2^2)), prototypes U[0,1),
last layer from the class identity; inputs resident in HBM before timing starts.

Also measured (second BASELINE metric, "push argmin ms/img"): the push of full-resolution
images (1024x2048 labels, 129x257 maps, P=190) through mask -> fused argmin -> merge.

Prints ONE JSON line (rank 0). Run: python bench.py [--gpus N --steps K --warmup W], or under
torch.distributed.run for N>1 (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from protoseg_amd import _lib  # noqa: E402
from protoseg_amd.distributed import init_from_env, world_info  # noqa: E402

PEAK_HBM_GBPS = 8000.0       # MI355X_MICROARCH.md chip table (spec)
PEAK_F32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector), spec
PEAK_F32_MFMA_TFLOPS = 157.3  # dense f32-input MFMA (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md
PEAK_BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA (spec, no sparsity), MI355X_MICROARCH.md
# Peak rate of f32-product FLOPs per precision mode: the bf16 split modes execute 3 or 6
# bf16 MFMA products per algorithmic f32 product (bf16_split.h).
PRODUCT_PEAK_TFLOPS = {"bf16x3": PEAK_BF16_MFMA_TFLOPS / 3, "bf16x6": PEAK_BF16_MFMA_TFLOPS / 6,
                       "f32": PEAK_F32_MFMA_TFLOPS}
SEED = 20220227


def baseline_metric() -> str:
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, KeyError, ValueError):
        return "training img/s (513x513, 19 prototypes/class) at 1/2/4/8 MI355X; push argmin ms/img"


class LayerStep:
    """Preallocated buffers + direct C-ABI launches (no per-step allocation)."""

    def __init__(self, B, C, h, w, P, K, x_dtype, device, seed, precision="bf16x3"):
        gen = torch.Generator(device="cpu").manual_seed(seed)
        self.B, self.C, self.h, self.w, self.P, self.K = B, C, h, w, P, K
        x = torch.sigmoid(2.0 * torch.randn(B, C, h, w, generator=gen))
        self.x = x.to(device=device, dtype=x_dtype).contiguous()
        self.protos = torch.rand(P, C, generator=gen).to(device)
        ident = torch.zeros(P, K)
        per = P // K
        for i in range(K):
            ident[i * per:(i + 1) * per, i] = 1
        self.w_last = (ident.t() * 1.5 - 0.5).contiguous().to(device)  # 1 own class, -0.5 else
        self.g_logits = (torch.randn(B, h, w, K, generator=gen) / (B * h * w)).to(device)
        f32 = dict(device=device, dtype=torch.float32)
        self.dist = torch.empty(B, P, h, w, **f32)
        self.logits = torch.empty(B, h, w, K, **f32)
        self.g_x = torch.empty_like(self.x)
        self.g_p = torch.empty(P, C, **f32)
        self.g_w = torch.empty(K, P, **f32)
        lib = _lib.load()
        self.ws_bytes = lib.protoseg_l2_bwd_workspace_size(B, C, h, w, P, K)
        self.ws = torch.empty(self.ws_bytes, device=device, dtype=torch.uint8)
        self.xdt = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.float16: _lib.F16}[x_dtype]
        self.device = device
        self.prec = _lib.PRECISIONS[precision]
        # The trained parameters (sharing storage with the kernels' buffers; the backward writes
        # their .grad in place) and the reference's optimizer (module.py:391: Adam; lr of the
        # prototype vectors, gin joint_optimizer_lr_prototype_vectors) on the HIP kernel
        # (protoseg_amd.optim.Adam: one launch for both tensors, step count on the device, so the
        # update runs inside the step's HIP graph).
        from protoseg_amd.optim import Adam
        self.params = [torch.nn.Parameter(self.protos), torch.nn.Parameter(self.w_last)]
        self.params[0].grad, self.params[1].grad = self.g_p, self.g_w
        # weight decay: gin joint_optimizer_weight_decay = 5e-4 (module.py:359-375 passes it to
        # every group but the prototype vectors'; one group here keeps one launch, same cost)
        self.opt = Adam(self.params, lr=2.5e-4, weight_decay=5e-4)
        self.buckets = None
        # one operand prep per step: the forward's prep launch also writes the backward's
        # operand images (protoseg_l2_fwd_ex), as the autograd op does in training
        # (PROTOSEG_FWD_OPERANDS=0: the backward prepares its own, for A/B)
        # the wide family's backward reads the forward's distances (protoseg_l2_bwd_saved), as the
        # autograd op does in training
        self.reads_dist = bool(lib.protoseg_l2_bwd_reads_dist(C, P, K, self.prec))
        nops = lib.protoseg_l2_train_operands_bytes(C, P, K, self.prec)
        if os.environ.get("PROTOSEG_FWD_OPERANDS", "1") == "0":
            nops = 0
        self.ops_bytes = nops
        self.ops = torch.empty(max(nops, 1), device=device, dtype=torch.uint8)
        # the optimizer step writes the next forward's operand images (protoseg_l2_adam_prep), so
        # the step is forward, backward (+ slab reduce) and update, with no prep launch
        # (PROTOSEG_FOLD_PREP=0: Adam and the forward's prep launch separately, for A/B)
        self.fold = (nops > 0 and os.environ.get("PROTOSEG_FOLD_PREP", "1") != "0"
                     and bool(lib.protoseg_l2_adam_prep_supported(C, P, K, self.prec)))
        self.ops_ready = False  # the operand block holds the current parameters' images

    def _stream(self):
        return _lib.stream_of(self.device)

    def _ops(self):
        return (_lib.ptr(self.ops) if self.ops_bytes else ctypes.c_void_p(None)), self.ops_bytes

    def fwd(self):
        act = _lib.ACT_LOG | (_lib.OPERANDS_READY if self.ops_ready else 0)
        _lib.call("protoseg_l2_fwd_ex", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w,
                  _lib.ptr(self.protos), self.P, _lib.ptr(self.w_last), self.K, 1e-4, act, self.prec,
                  _lib.ptr(self.dist), ctypes.c_void_p(None), _lib.ptr(self.logits), *self._ops(), self._stream())

    def bwd_x(self):
        _lib.call("protoseg_l2_bwd", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w, _lib.ptr(self.protos),
                  self.P, _lib.ptr(self.w_last), self.K, 1e-4, _lib.ACT_LOG, self.prec, _lib.ptr(self.g_logits),
                  ctypes.c_void_p(None), _lib.ptr(self.g_x), ctypes.c_void_p(None), ctypes.c_void_p(None),
                  ctypes.c_void_p(None), 0, self._stream())

    def bwd_pw(self):
        _lib.call("protoseg_l2_bwd", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w, _lib.ptr(self.protos),
                  self.P, _lib.ptr(self.w_last), self.K, 1e-4, _lib.ACT_LOG, self.prec, _lib.ptr(self.g_logits),
                  ctypes.c_void_p(None), ctypes.c_void_p(None), _lib.ptr(self.g_p), _lib.ptr(self.g_w),
                  _lib.ptr(self.ws), self.ws_bytes, self._stream())

    def bwd(self):
        """One backward call for g_x, g_prototypes and g_last_layer, as the autograd op makes it
        (ops.l2_backward), reading the operand images the forward's prep wrote (the wide family:
        the forward's distances)."""
        if self.reads_dist:
            _lib.call("protoseg_l2_bwd_saved", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w,
                      _lib.ptr(self.protos), self.P, _lib.ptr(self.w_last), self.K, 1e-4, _lib.ACT_LOG, self.prec,
                      _lib.ptr(self.dist), _lib.ptr(self.g_logits), ctypes.c_void_p(None), _lib.ptr(self.g_x),
                      _lib.ptr(self.g_p), _lib.ptr(self.g_w), _lib.ptr(self.ws), self.ws_bytes, self._stream())
            return
        _lib.call("protoseg_l2_bwd_ex", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w,
                  _lib.ptr(self.protos), self.P, _lib.ptr(self.w_last), self.K, 1e-4, _lib.ACT_LOG, self.prec,
                  _lib.ptr(self.g_logits), ctypes.c_void_p(None), _lib.ptr(self.g_x), _lib.ptr(self.g_p),
                  _lib.ptr(self.g_w), _lib.ptr(self.ws), self.ws_bytes, *self._ops(), self._stream())

    # ---- KLD training step (BASELINE configs[2], cityscapes_kld_imnet: loss_weight_kld = 0.25) ----
    def setup_kld(self, seed, weight=0.25):
        gen = torch.Generator(device="cpu").manual_seed(seed + 1)
        blocks = torch.randint(0, self.K + 1, (self.B, (self.h + 7) // 8, (self.w + 7) // 8), generator=gen)
        tgt = blocks.repeat_interleave(8, 1).repeat_interleave(8, 2)[:, :self.h, :self.w]
        self.target = tgt.reshape(self.B, -1).contiguous().to(self.device)  # resized labels, 0 = void
        per = self.P // self.K
        self.proto_class = torch.clamp(torch.arange(self.P) // per, max=self.K - 1).to(torch.int32).to(self.device)
        self.mpc = int(torch.bincount(self.proto_class.cpu().long()).max())
        lib = _lib.load()
        self.kld_ws_bytes = lib.protoseg_kld_workspace_size(self.B, self.P, self.h * self.w, self.K)
        self.kld_ws = torch.empty(self.kld_ws_bytes, device=self.device, dtype=torch.uint8)
        self.kld_loss = torch.empty((), device=self.device, dtype=torch.float32)
        self.kld_gloss = torch.full((), weight, device=self.device, dtype=torch.float32)
        self.g_dist = torch.empty_like(self.dist)
        n = self.B * self.h * self.w
        self.g_cls = torch.empty(n, self.mpc, device=self.device, dtype=torch.float32)
        self.pix_cls = torch.empty(n, device=self.device, dtype=torch.int32)
        self.proto_slot = torch.empty(self.P, device=self.device, dtype=torch.int32)

    def kld_fwd(self):
        _lib.call("protoseg_kld_forward", _lib.ptr(self.dist), self.B, self.P, self.h * self.w, _lib.ptr(self.target),
                  _lib.I64, _lib.ptr(self.proto_class), self.K, self.mpc, _lib.ptr(self.kld_loss), ctypes.c_void_p(None),
                  _lib.ptr(self.kld_ws), self.kld_ws_bytes, self._stream())

    def kld_bwd(self):
        _lib.call("protoseg_kld_backward", _lib.ptr(self.dist), self.B, self.P, self.h * self.w, _lib.ptr(self.target),
                  _lib.I64, _lib.ptr(self.proto_class), self.K, self.mpc, _lib.ptr(self.kld_gloss),
                  _lib.ptr(self.kld_ws), self.kld_ws_bytes, _lib.ptr(self.g_dist), self._stream())

    def kld_bwd_compact(self):
        """The KLD gradient in its compact per-pixel class-slot layout (no [B, P, H, W] tensor)."""
        _lib.call("protoseg_kld_backward_compact", _lib.ptr(self.dist), self.B, self.P, self.h * self.w,
                  _lib.ptr(self.target), _lib.I64, _lib.ptr(self.proto_class), self.K, self.mpc,
                  _lib.ptr(self.kld_gloss), _lib.ptr(self.kld_ws), self.kld_ws_bytes, _lib.ptr(self.g_cls),
                  _lib.ptr(self.pix_cls), _lib.ptr(self.proto_slot), self._stream())

    def bwd_kld(self):
        """Backward with the compact KLD gradient expanded in the kernels (protoseg_l2_bwd_kld)."""
        _lib.call("protoseg_l2_bwd_kld_ex", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w,
                  _lib.ptr(self.protos), self.P, _lib.ptr(self.w_last), self.K, 1e-4, _lib.ACT_LOG, self.prec,
                  _lib.ptr(self.g_logits), _lib.ptr(self.g_cls), _lib.ptr(self.pix_cls), _lib.ptr(self.proto_slot),
                  self.mpc, _lib.ptr(self.g_x), _lib.ptr(self.g_p), _lib.ptr(self.g_w), _lib.ptr(self.ws),
                  self.ws_bytes, *self._ops(), self._stream())

    def bwd_gd(self):
        """Backward with the KLD distance gradient (protoseg_l2_bwd g_dist)."""
        _lib.call("protoseg_l2_bwd_ex", _lib.ptr(self.x), self.xdt, self.B, self.C, self.h, self.w,
                  _lib.ptr(self.protos), self.P, _lib.ptr(self.w_last), self.K, 1e-4, _lib.ACT_LOG, self.prec,
                  _lib.ptr(self.g_logits), _lib.ptr(self.g_dist), _lib.ptr(self.g_x), _lib.ptr(self.g_p),
                  _lib.ptr(self.g_w), _lib.ptr(self.ws), self.ws_bytes, *self._ops(), self._stream())

    def opt_step(self):
        self.ops_ready = bool(self.fold and self.opt.layer_step_with_operands(self.params[0], self.params[1], self.ops,
                                                                              1e-4, _lib.ACT_LOG, self.prec))
        self.opt.step()  # the other parameters (none here: a no-op after the fused update)

    def exchange(self, world):
        """Data-parallel gradient exchange: the training step's GradientBuckets (bucketed RCCL
        all-reduce, averaged), the same class train.PatchClassificationStep uses."""
        if world > 1:
            if self.buckets is None:
                from protoseg_amd.distributed import GradientBuckets
                self.buckets = GradientBuckets(self.params, average=True)
                # the backward writes g_P / g_W straight into the exchange buffers (no copy)
                self.buckets.bind_grads()
                self.g_p, self.g_w = self.params[0].grad, self.params[1].grad
            self.buckets.allreduce()
            self.buckets.wait()

    @property
    def fused(self):
        """bf16x3 at C = 64: the training backward is one kernel (l2_bwd_wave.hip for P > 192,
        up to 384 prototypes per launch; l2_bwd_fused.hip at P <= 192); other precisions run
        the two-kernel backward."""
        return self.prec == _lib.PRECISIONS["bf16x3"] and self.C == 64

    def kernel_names(self):
        """Kernel families behind the step's timed calls. The library's timing hook matches a
        family prefix (l2_fwd -> l2_fwd_bf16_kernel or l2_fwd_kernel, whichever the shape and
        precision select) and reports the full name it bracketed; the backward call also runs
        the operand-image prep and slab-reduce kernels, outside the bracket (inside it when the
        call runs over prototype chunks: then the bracket spans all chunks)."""
        return ["l2_fwd", "l2_bwd"] if self.fused else ["l2_fwd", "l2_bwd_x", "l2_bwd_pw"]

    def timed_calls(self):
        return [self.fwd, self.bwd] if self.fused else [self.fwd, self.bwd_x, self.bwd_pw]

    # algorithmic work per call (unpadded P, K); layer_report divides by launches
    def work(self):
        n = self.B * self.h * self.w
        xb = self.x.element_size()
        mm = 2.0 * n * self.P * self.C
        last = 2.0 * n * self.P * self.K
        fwd = (mm + last + 2.0 * n * self.C, n * self.C * xb + n * self.P * 4 + n * self.K * 4)
        if self.fused:  # S, g_act, g_x, g_P, g_W: 3 distance-sized + 2 class-sized products
            return {"l2_fwd": fwd,
                    "l2_bwd": (3 * mm + 2 * last, n * self.C * xb + n * self.K * 4 + n * self.C * xb)}
        return {
            "l2_fwd": fwd,
            "l2_bwd_x": (2 * mm + last, n * self.C * xb + n * self.K * 4 + n * self.C * xb),
            "l2_bwd_pw": (2 * mm + 2 * last, n * self.C * xb + n * self.K * 4),
        }


def roofline_entry(flops, nbytes, seconds, precision="f32"):
    peak = PRODUCT_PEAK_TFLOPS[precision]
    t_mfma = flops / (peak * 1e12)
    t_hbm = nbytes / (PEAK_HBM_GBPS * 1e9)
    if t_mfma >= t_hbm:
        ach = flops / seconds / 1e12
        return {"bound": "mfma", "achieved": round(ach, 3), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(ach / peak, 4)}
    ach = nbytes / seconds / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBPS, 4)}


def pmc_traffic(kernel: str, config_key: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary, if one
    was collected for this exact configuration (profiles/pmc_traffic.json), else None."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            data = json.load(f)
        return data[config_key][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def capture(fn, stream):
    """HIP graph of fn()'s launches on `stream` (the C ABI launches on torch's current stream)."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        fn()
    return g


def time_layer(step: LayerStep, steps: int, warmup: int, world: int, use_graph: bool):
    """Times `steps` training steps of the prototype layer: forward, backward (g_x, g_P, g_W),
    [N > 1: the bucketed gradient all-reduce], Adam update of P and W.

    A step is the forward call and one backward call, as the autograd op issues them, then the
    optimizer. With use_graph the C-ABI calls and the (capturable) Adam update are captured into
    HIP graphs and replayed (no host launch gaps); at N > 1 the all-reduce runs between the
    backward graph and the optimizer graph. Per-kernel device times come from HIP events the
    library records around each launch of the named kernel during eager calls on the same stream."""
    names = step.kernel_names()
    calls = step.timed_calls()
    stream = torch.cuda.Stream(step.device)
    with torch.cuda.stream(stream):
        for _ in range(max(1, warmup)):
            for c in [step.fwd, step.bwd] + calls:
                c()
            step.exchange(world)
            step.opt_step()
        torch.cuda.synchronize()
        if use_graph and world == 1:
            g_step = capture(lambda: [step.fwd(), step.bwd(), step.opt_step()], stream)
            run_step = g_step.replay
        elif use_graph and os.environ.get("PROTOSEG_DP_CAPTURE", "1") == "1":
            # the whole step, RCCL all-reduce included, as one graph: the exchange is sync-free
            # (GradientBuckets: gradients are views into its buffers, no host reads)
            g_step = capture(lambda: [step.fwd(), step.bwd(), step.exchange(world), step.opt_step()], stream)
            run_step = g_step.replay
        elif use_graph:
            g_grad = capture(lambda: [step.fwd(), step.bwd()], stream)
            g_opt = capture(step.opt_step, stream)
            run_step = lambda: (g_grad.replay(), step.exchange(world), g_opt.replay())  # noqa: E731
        else:
            run_step = lambda: (step.fwd(), step.bwd(), step.exchange(world), step.opt_step())  # noqa: E731
        for _ in range(warmup):
            run_step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run_step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # per-kernel device time: the library records a start/stop event pair around each launch
        # of the one named kernel (protoseg_timing_events_n) in an eager call on this stream, so
        # the figure is the kernel alone, per dispatch, as rocprofv3 reports it (not the call's
        # prep / reduce launches; a prototype-chunked call yields one pair per chunk).
        lib = _lib.load()
        per_kernel = {n: [] for n in names}
        actual, launches = {}, {}
        npair = 8
        e = [[torch.cuda.Event(enable_timing=True) for _ in range(npair)] for _ in range(2)]
        for row in e:
            for ev in row:
                ev.record(stream)  # creates the HIP events
        torch.cuda.synchronize()
        starts = (ctypes.c_void_p * npair)(*[ev.cuda_event for ev in e[0]])
        stops = (ctypes.c_void_p * npair)(*[ev.cuda_event for ev in e[1]])
        for n, c in zip(names, calls):
            lib.protoseg_timing_events_n(n.encode(), starts, stops, npair)
            try:
                lib.protoseg_timing_launches()
                for _ in range(steps):
                    c()
                    torch.cuda.synchronize()
                    k = lib.protoseg_timing_launches()
                    if k < 1 or k > npair:
                        raise RuntimeError(f"timing hook bracketed {k} launches of {n}*")
                    launches[n] = k
                    per_kernel[n] += [e[0][i].elapsed_time(e[1][i]) * 1e-3 for i in range(k)]
                actual[n] = lib.protoseg_timing_kernel().decode()
                if not actual[n].startswith(n + "_"):
                    raise RuntimeError(f"timing hook did not bracket a {n}* kernel (got {actual[n]!r})")
            finally:
                lib.protoseg_timing_events_n(None, None, None, 0)
    step.launches = launches
    return elapsed, {n: float(np.mean(v)) for n, v in per_kernel.items()}, actual


def time_kld_step(step: LayerStep, steps: int, warmup: int, compact: bool = True):
    """BASELINE configs[2] step on one GPU: forward, KLD loss (module.py:167-208) forward and
    backward, layer backward with g_logits and the KLD gradient, Adam, as one HIP graph per step.
    compact: the KLD gradient in its per-pixel class-slot layout, expanded in the layer backward's
    kernels (what kld.kld_loss on PPNet's distances does); else the dense [B, P, H, W] g_dist.
    Returns ms per step and the per-launch event times of the two KLD calls."""
    kbwd = step.kld_bwd_compact if compact else step.kld_bwd
    calls = [step.fwd, step.kld_fwd, kbwd, step.bwd_kld if compact else step.bwd_gd, step.opt_step]
    stream = torch.cuda.Stream(step.device)
    with torch.cuda.stream(stream):
        for _ in range(max(1, warmup)):
            for c in calls:
                c()
        torch.cuda.synchronize()
        g = capture(lambda: [c() for c in calls], stream)
        g_kf, g_kb = capture(step.kld_fwd, stream), capture(kbwd, stream)
        for _ in range(warmup):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ms_f, ms_b = [], []
        for _ in range(steps):
            ev[0].record(stream)
            g_kf.replay()
            ev[1].record(stream)
            g_kb.replay()
            ev[2].record(stream)
            torch.cuda.synchronize()
            ms_f.append(ev[0].elapsed_time(ev[1]))
            ms_b.append(ev[1].elapsed_time(ev[2]))
    loss = float(step.kld_loss)
    n = step.B * step.h * step.w
    kb = float(np.mean(ms_b)) * 1e-3
    out = {"workload": "cityscapes_kld_imnet step on 1 GPU: fwd + KLD fwd/bwd (loss_weight_kld 0.25) + bwd with the "
                       + ("compact KLD gradient (protoseg_l2_bwd_kld)" if compact else "dense g_dist") + " + Adam update",
           "ms_per_step": round(elapsed / steps * 1e3, 4), "img_per_s": round(step.B * steps / elapsed, 1),
           "kld_forward_ms": round(float(np.mean(ms_f)), 4), "kld_backward_ms": round(kb * 1e3, 4),
           "loss": round(loss, 6), "prototypes": step.P}
    if not compact:
        out["kld_backward_gbps"] = round(n * step.P * 4 / kb / 1e9, 1)
    return out


def time_sigmoid_step(step: LayerStep, steps: int, warmup: int):
    """The add-on's nn.Sigmoid (model.py:124-128) in the training step at the headline shape:
    (a) fused into the layer kernels' x load (PROTOSEG_X_SIGMOID: the step's input is the
    pre-activation, the backward returns its gradient), against (b) the unfused step: sigmoid
    forward, the layer step on sigmoid(X), sigmoid backward (torch's elementwise kernels).
    Both as one HIP graph per step with the Adam update; returns ms per step of each."""
    gen = torch.Generator(device="cpu").manual_seed(7)
    pre = (2.0 * torch.randn(step.x.shape, generator=gen)).to(step.device, step.x.dtype)
    g_pre = torch.empty_like(pre)
    sig = torch.empty_like(pre)
    null = ctypes.c_void_p(None)
    act_f = _lib.ACT_LOG | _lib.X_SIGMOID

    def common(x, act, gx):
        _lib.call("protoseg_l2_fwd_ex", _lib.ptr(x), step.xdt, step.B, step.C, step.h, step.w,
                  _lib.ptr(step.protos), step.P, _lib.ptr(step.w_last), step.K, 1e-4, act, step.prec,
                  _lib.ptr(step.dist), null, _lib.ptr(step.logits), *step._ops(), step._stream())
        _lib.call("protoseg_l2_bwd_ex", _lib.ptr(x), step.xdt, step.B, step.C, step.h, step.w,
                  _lib.ptr(step.protos), step.P, _lib.ptr(step.w_last), step.K, 1e-4, act, step.prec,
                  _lib.ptr(step.g_logits), null, _lib.ptr(gx), _lib.ptr(step.g_p), _lib.ptr(step.g_w),
                  _lib.ptr(step.ws), step.ws_bytes, *step._ops(), step._stream())
        step.opt_step()

    def fused():
        common(pre, act_f, g_pre)

    def unfused():
        torch.sigmoid(pre, out=sig)
        common(sig, _lib.ACT_LOG, step.g_x)
        torch.ops.aten.sigmoid_backward(step.g_x, sig, grad_input=g_pre)

    out = {}
    stream = torch.cuda.Stream(step.device)
    with torch.cuda.stream(stream):
        for name, fn in (("fused_on_load", fused), ("separate_sigmoid", unfused)):
            for _ in range(max(1, warmup)):
                fn()
            torch.cuda.synchronize()
            g = capture(fn, stream)
            for _ in range(warmup):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                g.replay()
            torch.cuda.synchronize()
            out[name + "_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 4)
    out["workload"] = (f"layer training step incl. the add-on sigmoid, P={step.P}: fused into the x load "
                       f"(PROTOSEG_X_SIGMOID) vs sigmoid fwd/bwd as separate HBM passes")
    return out


def host_cores():
    """CPUs this process may run on (the cpuset / affinity mask; os.cpu_count() is the whole
    machine) and the cgroup CPU quota in cores if one is set (None otherwise)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cores = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return cores, quota


def cpu_layer_baseline(B, C, h, w, P, K, warmup=3, reps=10):
    """Oracle (op-for-op torch-CPU restatement of model.py:203-283 + autograd) fwd+bwd of one
    step's batch, on every host core this process may use (3 warm-up + 10 timed
    reps, median)."""
    from oracle import protoseg_oracle as po
    cores, quota = host_cores()
    # threads = the cores this process actually gets: the affinity mask, capped by the cgroup
    # CPU quota when one is set (on the GPU box the quota is 16 of 256 visible CPUs; 256 torch
    # threads there oversubscribe the quota and ran 80x slower, 7.9 s per step).
    threads = min(cores, max(1, math.ceil(quota))) if quota else cores
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    x, protos, w_last = po.synthetic_inputs(B, C, h, w, P, K, SEED)
    g = torch.randn(B, h, w, K, generator=torch.Generator().manual_seed(SEED))
    for _ in range(warmup):
        po.forward_backward(x, protos, w_last, g, None)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        po.forward_backward(x, protos, w_last, g, None)
        times.append(time.perf_counter() - t0)
    torch.set_num_threads(prev)
    med = float(np.median(times))
    return {"value": round(B / med, 3), "unit": "img/s", "cores": threads, "kind": "port",
            "sample": f"{warmup} warm-up + {reps} timed reps (median {med * 1e3:.1f} ms) of the oracle fwd+bwd "
                      f"(torch-CPU restatement of model.py:203-283 + autograd) over one step's batch "
                      f"{B}x{C}x{h}x{w}, P={P}, K={K}; torch threads = {threads} = the process's CPUs "
                      f"(affinity {cores}, os.cpu_count() {os.cpu_count()}) capped by the cgroup quota ({quota} cores)"}


def make_push_inputs(n_img, C, H, W, h, w, P, K, device, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.sigmoid(2.0 * torch.randn(n_img, C, h, w, generator=gen)).to(device)
    protos = torch.rand(P, C, generator=gen).to(device)
    rng = np.random.default_rng(seed)
    blocks = rng.integers(0, K + 1, size=(n_img, H // 16, W // 16)).astype(np.uint8)
    labels = torch.from_numpy(np.repeat(np.repeat(blocks, 16, 1), 16, 2)).to(device)
    pc = (torch.arange(P) // (P // K)).to(torch.int32).to(device)
    return x, protos, labels, pc


def kernel_launch_times(name, fn, reps, npair=8, actual=None):
    """Per-launch device seconds of the kernel `name` (a family prefix) over `reps` eager calls of
    fn(), from the library's per-launch event hook (protoseg_timing_events_n). Returns (mean s per
    launch, launches per call); `actual` (a list) receives the full name of the kernel bracketed."""
    lib = _lib.load()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(npair)] for _ in range(2)]
    for row in ev:
        for e in row:
            e.record()
    torch.cuda.synchronize()
    starts = (ctypes.c_void_p * npair)(*[e.cuda_event for e in ev[0]])
    stops = (ctypes.c_void_p * npair)(*[e.cuda_event for e in ev[1]])
    times, per_call = [], 0
    lib.protoseg_timing_events_n(name.encode(), starts, stops, npair)
    try:
        lib.protoseg_timing_launches()
        for _ in range(reps):
            fn()
            torch.cuda.synchronize()
            k = lib.protoseg_timing_launches()
            if k < 1 or k > npair:
                raise RuntimeError(f"timing hook bracketed {k} launches of {name}")
            per_call = k
            times += [ev[0][i].elapsed_time(ev[1][i]) * 1e-3 for i in range(k)]
        if actual is not None:
            actual.append(lib.protoseg_timing_kernel().decode())
    finally:
        lib.protoseg_timing_events_n(None, None, None, 0)
    return float(np.mean(times)), per_call


def time_push(n_img, steps, warmup, device, C=64, H=1024, W=2048, h=129, w=257, P=190, K=19, scan_images=64):
    """The shipped push driver's inner step (push.push_update, one call per batch of n_img
    equal-geometry images, as push_prototypes issues it with images_per_batch = n_img):
    patch mask -> top-2 argmin -> strict-'<' merge. One timed step is a SCAN of `scan_images`
    DISTINCT images (scan_images / n_img batches, first_img advancing) from a fresh running state,
    as push_prototypes walks dataset.img_ids (push.py:101): the argmin's skip of candidates above
    the running runner-up sees what a real scan sees, never images it has already merged. Wall
    time per image over `steps` scans; the argmin kernel's per-launch device time from the
    library's event hook over one scan."""
    from protoseg_amd import push as dpush
    nb = max(1, scan_images // n_img)
    batches = [make_push_inputs(n_img, C, H, W, h, w, P, K, device, SEED + 1000 * i) for i in range(nb)]
    pc = batches[0][3]
    protos = batches[0][1]  # one set of prototypes for the whole scan
    words = dpush.mask_words(K)  # push_prototypes computes it once per push (no per-call host sync)
    states = [dpush.PushState.create(P, C, device) for _ in range(steps + warmup + 1)]

    def scan(state):
        for i, (x, _, labels, _) in enumerate(batches):
            dpush.push_update(state, x, labels, protos, pc, i * n_img, words=words)

    for i in range(warmup):
        scan(states[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        scan(states[warmup + i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kname = []
    argmin_s, launches = kernel_launch_times("push_argmin", lambda: scan(states[-1]), 1, npair=2 * nb, actual=kname)
    launches_per_call = launches // nb
    argmin_call = argmin_s * launches_per_call
    flops = 2.0 * n_img * h * w * P * C
    nbytes = n_img * (C * h * w * 4 + h * w * 4)  # x read once + the u32 patch mask
    return {"ms_per_img": round(elapsed / (steps * nb * n_img) * 1e3, 4), "images_per_call": n_img,
            "workload": f"push_prototypes inner step (push_update: mask+top-2 argmin+merge), a scan of {nb * n_img} "
                        f"distinct images from a fresh state, labels {H}x{W} u8, map {C}x{h}x{w} f32, P={P}, K={K}",
            "argmin_kernel_ms_per_img": round(argmin_call / n_img * 1e3, 4),
            "argmin_launches_per_call": launches_per_call,
            # the argmin computes on bf16 MFMA with exact three-term splits (bf16x6: six products per
            # f32 multiply-add), so its peak is the bf16 dense peak / 6; the flops are the algorithmic
            # 2*P*C per pixel, including the candidates the runner-up bound lets it skip (an
            # effective rate); f32_mfma_frac prices the same rate against the f32 MFMA peak
            "roofline": (lambda r: r | {"kernel": kname[0] if kname else "push_argmin", "arith": "bf16x6",
                                        "f32_mfma_frac": round(r["achieved"] / PEAK_F32_MFMA_TFLOPS, 4)
                                        if r["unit"] == "TFLOP/s" else None})(
                roofline_entry(flops / launches_per_call, nbytes / launches_per_call, argmin_s, "bf16x6"))}


def cpu_push_baseline(budget_s, C=64, H=1024, W=2048, h=129, w=257, P=190, K=19):
    """Oracle restatement of push.py:184-281 on one image, op for op as the reference runs it on
    the CPU: distances (torch-CPU conv, model.py:203-221), the label map as a torch.LongTensor
    with one `.item()` per pixel for the class -> patch sets (push.py:186, 214-230), then the
    per-prototype Python argmin (push.py:235-281). Single thread."""
    from oracle import protoseg_oracle as po
    from oracle import push_oracle as pu
    x, protos, labels, pc = make_push_inputs(1, C, H, W, h, w, P, K, "cpu", SEED)
    lab = labels[0].numpy()
    n, t0 = 0, time.perf_counter()
    while True:
        d = po.l2_convolution(x, protos[:, :, None, None], torch.ones(P, C, 1, 1))[0]
        st = pu.PushOracleState(P, C)
        sets = pu.class_to_patch_index_dict_torch(lab, h, w, K)
        pu.update_prototypes_on_image_core(st, x[0].numpy(), d.permute(1, 2, 0).numpy(), lab, pc.numpy(), K, 0,
                                           sets=sets)
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"ms_per_img": round(dt / n * 1e3, 1), "cores": 1, "kind": "port",
            "sample": f"{n} image(s): push.py:184-281 on the CPU as the reference runs it (torch.LongTensor labels, "
                      f"per-pixel .item() patch sets, per-prototype argmin), {H}x{W} labels, {C}x{h}x{w} map, P={P}"}


def _timed_calls(run, steps, warmup):
    """Runs run(ev) `steps` times after `warmup`; returns (wall s per call, mean event s per call
    of the bracketed kernel). Events are recorded on torch's current stream, which is the stream
    the C ABI launches on."""
    for _ in range(warmup):
        run(None)
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
    t0 = time.perf_counter()
    for s in range(steps):
        run(evs[s])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    return wall, float(np.mean([e[0].elapsed_time(e[1]) for e in evs])) * 1e-3


def time_knn(n_img, steps, warmup, device, H=1024, W=2048, h=129, w=257, P=190, K=19, k=5):
    """k-NN search (find_nearest.py:87-230) over batches of push_forward distance maps: label
    resize -> masked f64 image minima -> patch labels -> heap push. The dominant kernel
    (knn_image_min_kernel) streams the [n, P, h, w] f32 maps once: algorithmic bytes = maps +
    the int32 small labels."""
    from protoseg_amd import knn as dknn
    gen = torch.Generator().manual_seed(SEED + 3)
    dmaps = (torch.rand(n_img, P, h, w, generator=gen) * 40).to(device)
    rng = np.random.default_rng(SEED + 3)
    blocks = rng.integers(0, K + 1, size=(n_img, H // 16, W // 16)).astype(np.uint8)
    labels = torch.from_numpy(np.repeat(np.repeat(blocks, 16, 1), 16, 2)).to(device)
    pc = (torch.arange(P) // (P // K)).to(torch.int32).to(device)
    state = dknn.KnnState.create(P, k, device)
    small = torch.empty((n_img, h, w), device=device, dtype=torch.int32)
    min_dist = torch.empty((n_img, P), device=device, dtype=torch.float64)
    min_idx = torch.empty((n_img, P), device=device, dtype=torch.int32)
    plab = torch.empty((n_img, P), device=device, dtype=torch.int32)
    stream = _lib.stream_of(device)
    null = ctypes.c_void_p(None)

    def run(ev):
        _lib.call("protoseg_resize_label", _lib.ptr(labels), _lib.U8, n_img, H, W, h, w, null, 0, _lib.ptr(small),
                  stream)
        if ev is not None:
            ev[0].record()
        _lib.call("protoseg_knn_image_min", _lib.ptr(dmaps), n_img, P, h, w, _lib.ptr(small), _lib.ptr(min_dist),
                  _lib.ptr(min_idx), stream)
        if ev is not None:
            ev[1].record()
        _lib.call("protoseg_knn_patch_label", _lib.ptr(min_idx), n_img, P, h, w, _lib.ptr(labels), _lib.U8, H, W,
                  null, 0, _lib.ptr(pc), _lib.ptr(plab), _lib.ptr(state.status), stream)
        _lib.call("protoseg_knn_heap_push", _lib.ptr(min_dist), _lib.ptr(min_idx), _lib.ptr(plab), n_img, 0, P, k,
                  _lib.ptr(state.neg), _lib.ptr(state.label), _lib.ptr(state.patch), _lib.ptr(state.img),
                  _lib.ptr(state.size), stream)

    wall, kern = _timed_calls(run, steps, warmup)
    nbytes = n_img * (P * h * w * 4 + h * w * 4)
    return {"ms_per_img": round(wall / n_img * 1e3, 4), "images_per_call": n_img, "k": k,
            "workload": f"k-NN search: labels {H}x{W} u8, maps {P}x{h}x{w} f32, K={K}",
            "image_min_kernel_ms_per_img": round(kern / n_img * 1e3, 4),
            "roofline": roofline_entry(0.0, nbytes, kern) | {"kernel": "knn_image_min_kernel"}}


def time_eval(n_img, steps, warmup, device, H=1024, W=2048, h=129, w=257, P=190, K=19):
    """mIoU evaluation counts (eval_valid.py:159-197) at Cityscapes eval resolution: bilinear
    upsample + argmax of K logits + argmin of P distances per output pixel, fused. Algorithmic
    bytes = the low-resolution logits and distances + the u8 labels (each read once)."""
    gen = torch.Generator().manual_seed(SEED + 5)
    logits = (torch.randn(n_img, h, w, K, generator=gen) * 3).to(device)
    dmaps = (torch.rand(n_img, P, h, w, generator=gen) * 40).to(device)
    rng = np.random.default_rng(SEED + 5)
    blocks = rng.integers(0, K + 1, size=(n_img, H // 16, W // 16)).astype(np.uint8)
    anns = torch.from_numpy(np.repeat(np.repeat(blocks, 16, 1), 16, 2)).to(device)
    pc = (torch.arange(P) // (P // K)).to(torch.int32).to(device)
    counts = torch.zeros(2 + 2 * K + P, device=device, dtype=torch.int64)
    stream = _lib.stream_of(device)
    null = ctypes.c_void_p(None)

    def run(ev):
        if ev is not None:
            ev[0].record()
        _lib.call("protoseg_eval_counts", _lib.ptr(logits), _lib.ptr(dmaps), n_img, h, w, K, P, _lib.ptr(anns),
                  _lib.U8, H, W, null, 0, _lib.ptr(pc), _lib.ptr(counts), stream)
        if ev is not None:
            ev[1].record()

    wall, kern = _timed_calls(run, steps, warmup)
    nbytes = n_img * ((K + P) * h * w * 4 + H * W)
    # VALU-bound: per output pixel and class/prototype, torch's bilinear form
    # h0*(w0*v00 + w1*v01) + h1*(w0*v10 + w1*v11) (6 mul + 3 add) and one compare = 10 flops,
    # against the f32 vector peak; the HBM figure is reported beside it.
    flops = n_img * 10.0 * (K + P) * H * W
    valu = flops / kern / 1e12
    hbm = roofline_entry(0.0, nbytes, kern)
    return {"ms_per_img": round(wall / n_img * 1e3, 4), "images_per_call": n_img,
            "workload": f"eval counts: labels {H}x{W} u8, logits {h}x{w}x{K}, distances {P}x{h}x{w} f32",
            "roofline": {"bound": "valu", "achieved": round(valu, 2), "peak": PEAK_F32_VALU_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(valu / PEAK_F32_VALU_TFLOPS, 4),
                         "hbm_gbps": hbm["achieved"], "hbm_frac": hbm["frac"], "kernel": "eval_rows_kernel"}}


def time_bound_boxes(steps, warmup, device, H=1024, W=2048, h=129, w=257, P=190, K=19):
    """Push post-step, high-activation bound boxes of all P prototypes (push.py:309-343) in one
    act_upsample + bound_boxes pair. The roofline line is the upsample, an HBM-write stream
    (cubic_upsample4_kernel at W % 4 == 0): algorithmic bytes = P * H * W * 4 (upsampled maps
    written once) + the P low-res activation maps read. bound_boxes_ms is the percentile select
    (two full reads of the maps) and the greedy walk."""
    from protoseg_amd import push as dpush
    gen = torch.Generator().manual_seed(SEED + 7)
    dmaps = (torch.rand(P, h, w, generator=gen) * 6).to(device)
    rng = np.random.default_rng(SEED + 7)
    blocks = rng.integers(0, K + 1, size=(1, H // 16, W // 16)).astype(np.uint8)
    labels = torch.from_numpy(np.repeat(np.repeat(blocks, 16, 1), 16, 2)).to(device)
    tc = (torch.arange(P) // (P // K)).to(torch.int32).to(device)
    r, c = rng.integers(0, h, P), rng.integers(0, w, P)
    rf = torch.as_tensor(np.stack([r * H // h, r * H // h + 9, c * W // w, c * W // w + 9], 1).astype(np.int32),
                         device=device)
    act = torch.empty_like(dmaps)
    up = torch.empty((P, H, W), device=device, dtype=torch.float32)
    thr = torch.empty(P, device=device, dtype=torch.float32)
    box = torch.empty((P, 4), device=device, dtype=torch.int32)
    stream = _lib.stream_of(device)
    null = ctypes.c_void_p(None)
    t_box = []

    def run(ev):
        if ev is not None:
            ev[0].record()
        _lib.call("protoseg_act_upsample", _lib.ptr(dmaps), P, h, w, H, W, _lib.ACT_LOG, 1e-4, float(64),
                  _lib.ptr(act), _lib.ptr(up), stream)
        if ev is not None:
            ev[1].record()
        _lib.call("protoseg_bound_boxes", _lib.ptr(up), P, H, W, _lib.ptr(labels), _lib.U8, 1, null, null, 0,
                  _lib.ptr(tc), _lib.ptr(rf), 95.0, 5, _lib.ptr(thr), _lib.ptr(box), stream)

    wall, kern = _timed_calls(run, steps, warmup)
    nbytes = P * (H * W * 4 + h * w * 4)
    return {"ms_per_push": round(wall * 1e3, 4), "prototypes": P,
            "workload": f"bound boxes: {P} maps {h}x{w} -> {H}x{W} cubic, 95th percentile, greedy crop",
            "act_upsample_ms": round(kern * 1e3, 4), "bound_boxes_ms": round((wall - kern) * 1e3, 4),
            "roofline": roofline_entry(0.0, nbytes, kern) | {"kernel": "act_kernel + cubic_upsample4_kernel"}}


def layer_report(step: LayerStep, per_kernel, actual, args):
    """Roofline of the step's dominant kernel (event-timed, algorithmic work per launch) and the
    per-kernel table."""
    # per launch: a prototype-chunked call runs its kernel once per chunk (near-equal chunks)
    launches = getattr(step, "launches", {})
    work = {n: (f / launches.get(n, 1), b / launches.get(n, 1)) for n, (f, b) in step.work().items()}
    dominant = max(per_kernel, key=lambda n: per_kernel[n] * launches.get(n, 1))
    flops, nbytes = work[dominant]
    prec = args.precision if "_bf16" in actual[dominant] else "f32"  # the family that ran
    roof = roofline_entry(flops, nbytes, per_kernel[dominant], prec)
    config_key = (f"B{step.B}_C{step.C}_{step.h}x{step.w}_P{step.P}_K{step.K}"
                  f"_{args.x_dtype}_{args.precision}")
    roof["traffic"] = pmc_traffic(actual[dominant], config_key)
    roof["kernel"] = actual[dominant]
    kernels = {}
    for n, s in per_kernel.items():
        f, b = work[n]
        kernels[actual[n]] = {"ms": round(s * 1e3, 4), "launches_per_call": launches.get(n, 1),
                              "tflops": round(f / s / 1e12, 2), "gbps": round(b / s / 1e9, 1)}
    return roof, kernels


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` outside a launcher: start N ranks (one process per GPU) with
    torch.distributed.run on 127.0.0.1 and return its exit code. Runs before anything touches the
    GPU; the children are started as child processes (never exec'd over this one)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def cpu_smoke(args, rank, world):
    """--cpu-smoke: the multi-rank plumbing without a GPU (gloo): every rank runs `steps` of the
    DP exchange of the layer step (GradientBuckets over g_P and g_W, CPU tensors of the headline
    shapes) between the same barriers as the GPU bench, rank 0 prints the JSON line. The value is
    the exchange rate only, labelled as such — it is a launcher test, not a measurement."""
    from protoseg_amd.distributed import GradientBuckets
    P, C, K = args.protos, args.channels, args.classes
    params = [torch.nn.Parameter(torch.rand(P, C)), torch.nn.Parameter(torch.rand(K, P))]
    buckets = GradientBuckets(params, average=True)
    for p in params:
        p.grad = torch.full_like(p, float(rank + 1))
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        buckets.allreduce()
        buckets.wait()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    mean_rank = float(params[0].grad[0, 0])  # mean of 1..world after averaging (idempotent)
    if rank == 0:
        print(json.dumps({"metric": "cpu-smoke: DP gradient exchange only (no GPU)", "value":
                          round(args.batch * world * args.steps / elapsed, 1), "unit": "img/s", "n_gpus": world,
                          "steps": args.steps, "warmup": 0, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                          "data": "synthetic", "config": {"workload": "cpu-smoke", "parallelism": f"dp{world}",
                                                          "backend": dist.get_backend() if world > 1 else None,
                                                          "grad_mean_check": mean_rank}}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def time_wide(device, B, C, h, w, P, K, x_dtype, steps=10, warmup=3, label="", precision="bf16x3"):
    """The layer step on the wide family (l2_wide.hip: any C / K, exact f32 MFMA GEMMs with fused
    epilogues): BASELINE configs[4]'s DenseNet depth and the reference's own construct_PPNet default
    (model.py:394). Whole fwd / bwd calls are event-timed (each is a chain of GEMM launches); the
    roofline is the call's algorithmic FLOPs against the product peak of the precision (bf16x3:
    2.5 PF / 3 on v_mfma_f32_32x32x16_bf16; f32: v_mfma_f32_32x32x2_f32)."""
    step = LayerStep(B, C, h, w, P, K, x_dtype, device, SEED, precision)
    stream = torch.cuda.Stream(device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_f, t_b = [], []
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            step.fwd()
            step.bwd()
            step.opt_step()
        torch.cuda.synchronize()
        g = capture(lambda: [step.fwd(), step.bwd(), step.opt_step()], stream)
        for _ in range(warmup):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        for _ in range(steps):
            ev[0].record(stream)
            step.fwd()
            ev[1].record(stream)
            step.bwd()
            ev[2].record(stream)
            torch.cuda.synchronize()
            t_f.append(ev[0].elapsed_time(ev[1]) * 1e-3)
            t_b.append(ev[1].elapsed_time(ev[2]) * 1e-3)
    n = B * h * w
    mm, last = 2.0 * n * P * C, 2.0 * n * P * K
    f_fwd = mm + last                # S, logits
    # g_act, g_x, g_P, g_W (+ S recomputed unless the backward reads the forward's distances)
    f_bwd = (2 if step.reads_dist else 3) * mm + 2 * last
    tf, tb = float(np.median(t_f)), float(np.median(t_b))
    prod = ("bf16x3 products on v_mfma_f32_32x32x16_bf16" if precision == "bf16x3"
            else "f32 products on v_mfma_f32_32x32x2_f32")
    peak = PRODUCT_PEAK_TFLOPS["bf16x3" if precision == "bf16x3" else "f32"]
    out = {"workload": label + f" (B={B}, C={C}, {h}x{w} map, P={P}, K={K}, {prod})",
           "img_per_s": round(B * steps / elapsed, 1), "ms_per_step": round(elapsed / steps * 1e3, 4),
           "fwd_ms": round(tf * 1e3, 4), "bwd_ms": round(tb * 1e3, 4)}
    for name, f, t in (("fwd", f_fwd, tf), ("bwd", f_bwd, tb)):
        ach = f / t / 1e12
        out[f"roofline_{name}"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(peak, 1),
                                   "unit": "TFLOP/s", "frac": round(ach / peak, 4)}
    del step
    return out


def time_small_batches(args, device, batches=(2, 4), protos=(361, 190), kld=True):
    """The layer step at the reference's per-GPU micro-batches (gin joint_batch_size = 2;
    configs[2]: 32 images over 8 GPUs = 4 per GPU), where launch and tail costs dominate; each
    with the KLD step (module.py:167-208 runs on every micro-step of configs[2]) beside it."""
    x_dtype = torch.float32 if args.x_dtype == "f32" else torch.bfloat16
    out = {}
    for P in protos:
        for B in batches:
            s = LayerStep(B, args.channels, args.fmap, args.fmap, P, args.classes, x_dtype, device, SEED,
                          args.precision)
            e, k, a = time_layer(s, args.steps, args.warmup, 1, args.launch == "graph")
            line = {"img_per_s": round(B * args.steps / e, 1), "ms_per_step": round(e / args.steps * 1e3, 4),
                    "kernels_ms": {a[n]: round(v * 1e3, 4) for n, v in k.items()}}
            if kld and not args.no_kld:
                # the KLD step at the drop-in's own micro-batch (cityscapes_kld_imnet.gin:23 / configs[2])
                s.setup_kld(SEED)
                kl = time_kld_step(s, max(5, args.steps // 2), 3)
                line["kld_step"] = {key: kl[key] for key in ("ms_per_step", "kld_forward_ms", "kld_backward_ms")}
                line["kld_step"]["ratio_to_plain_step"] = round(kl["ms_per_step"] / line["ms_per_step"], 3)
            out[f"B{B}_P{P}"] = line
            del s
    return out


def time_train_step(args, device, rank, world, accumulations=1, warm_accumulations=1, batch=4, P=190):
    """BASELINE configs[2] (cityscapes_kld_imnet.gin) end to end, data-parallel: PPNet on the
    in-tree DeepLabV2-ResNet101 (random init; deeplab_n_features 64, scales [], deeplab_simple
    add-on), synthetic 513x513 batches of `batch` images per GPU with 19-class labels (0 = void),
    train.PatchClassificationStep (module.py:118-243): cross entropy + KLD (0.25) + L1, loss /
    iter_size backward, every iter_size = 5 micro-steps the bucketed RCCL all-reduce of the whole
    gradient (GradientBuckets, launched from the backward's hooks) and the joint-phase Adam
    (module.py:357-391, weight decay 5e-4) on the HIP kernel. Times `accumulations` optimizer
    steps (x iter_size micro-steps) after `warm_accumulations`, between barriers; max over ranks."""
    from protoseg_amd.deeplab import deeplabv2_resnet101_features
    from protoseg_amd.model import construct_PPNet
    from protoseg_amd.optim import Adam
    from protoseg_amd.train import PatchClassificationStep, joint_param_groups
    iter_size = 5
    torch.manual_seed(SEED)  # identical initial weights on every rank
    feats = deeplabv2_resnet101_features(pretrained=False, deeplab_n_features=64, scales=[])
    net = construct_PPNet(img_size=513, prototype_shape=(P, 64, 1, 1), num_classes=args.classes,
                          prototype_activation_function="log", add_on_layers_type="deeplab_simple",
                          features=feats, bottleneck_stride=1, patch_classification=True).to(device)
    net.train()
    net.features.base.freeze_bn()  # module.py:127
    opt = Adam(joint_param_groups(net))
    step = PatchClassificationStep(net, opt, loss_weight_kld=0.25, loss_weight_l1=1e-4, iter_size=iter_size)
    grad_mb = sum(p.numel() * p.element_size() for p in step.buckets.params) / 2 ** 20
    gen = torch.Generator().manual_seed(SEED + 11 + rank)
    images = torch.randn(iter_size, batch, 3, 513, 513, generator=gen).to(device)
    blocks = torch.randint(0, args.classes + 1, (iter_size, batch, 33, 33), generator=gen)
    targets = blocks.repeat_interleave(16, 2).repeat_interleave(16, 3)[:, :, :513, :513].contiguous().to(device)

    def run(n_acc):
        for _ in range(n_acc):
            for i in range(iter_size):
                step(images[i], targets[i])

    run(warm_accumulations)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run(accumulations)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    micro = accumulations * iter_size
    return {"workload": "cityscapes_kld_imnet DP training step: DeepLabV2-R101 (PyTorch-ROCm) + prototype layer and "
                        "KLD (HIP) + bucketed RCCL gradient all-reduce + HIP Adam, synthetic 513x513",
            "img_per_s": round(world * batch * micro / elapsed, 2), "n_gpus": world, "per_gpu_batch": batch,
            "global_batch": world * batch, "iter_size": iter_size, "prototypes": P,
            "ms_per_micro_step": round(elapsed / micro * 1e3, 2),
            "ms_per_optimizer_step": round(elapsed / accumulations * 1e3, 2),
            "micro_steps_timed": micro, "grad_exchange_mb": round(grad_mb, 1),
            "buckets": len(step.buckets.buckets), "backbone_dtype": "f32",
            "dominated_by": "the DeepLabV2-ResNet101 backbone (PyTorch-ROCm / MIOpen convolutions, outside this "
                            "framework's scope), not the prototype layer: at 513x513 MIOpen picks GemmFwdRest / "
                            "GemmBwdRest / GemmWrwUniversal solvers that ask for more workspace than it grants and "
                            "fall back, so this line measures the backbone; the layer's own cost is the headline "
                            "metric and the kld_step line"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU per step")
    ap.add_argument("--protos", type=int, default=361, help="19 prototypes/class x 19 classes (the metric)")
    ap.add_argument("--side-protos", type=int, default=190, help="side line: cityscapes_*_imnet.gin (10/class); 0 = off")
    ap.add_argument("--classes", type=int, default=19)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--fmap", type=int, default=65, help="feature-map side (513 crop -> 65)")
    ap.add_argument("--x-dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--precision", choices=["bf16x3", "bf16x6", "f32"], default="bf16x3",
                    help="product arithmetic of the prototype layer (bf16_split.h)")
    ap.add_argument("--push-images", type=int, default=8)
    ap.add_argument("--push-steps", type=int, default=5)
    ap.add_argument("--no-push", action="store_true")
    ap.add_argument("--no-f32-line", action="store_true", help="skip the exact-f32 side line")
    ap.add_argument("--no-kld", action="store_true")
    ap.add_argument("--no-knn", action="store_true")
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="push CPU baseline time budget")
    ap.add_argument("--launch", choices=["graph", "eager"], default="graph",
                    help="graph: each step is one HIP graph replay of the three C-ABI calls")
    ap.add_argument("--no-small-batch", action="store_true", help="skip the B=2/4 side lines")
    ap.add_argument("--no-wide", action="store_true", help="skip the wide-family (C=1024 / C=512, P=2000) side lines")
    ap.add_argument("--no-sigmoid", action="store_true", help="skip the fused add-on sigmoid side line")
    ap.add_argument("--no-train", action="store_true", help="skip the DeepLabV2-R101 DP training-step side line")
    ap.add_argument("--train-accumulations", type=int, default=1,
                    help="optimizer steps (x iter_size 5 micro-steps) timed in the training side line")
    ap.add_argument("--cpu-smoke", action="store_true",
                    help="no GPU: launch the ranks and time only the gloo gradient exchange (launcher test)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the N ranks here, before any GPU call, and report theirs
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.cpu_smoke:
        cpu_smoke(args, *init_from_env("gloo")[::2])
        return

    rank, local_rank, world = init_from_env()
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    device = torch.device(f"cuda:{local_rank}")
    torch.cuda.set_device(device)
    x_dtype = torch.float32 if args.x_dtype == "f32" else torch.bfloat16

    step = LayerStep(args.batch, args.channels, args.fmap, args.fmap, args.protos, args.classes, x_dtype, device,
                     SEED + rank, args.precision)
    elapsed, per_kernel, actual = time_layer(step, args.steps, args.warmup, world, args.launch == "graph")
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    images = args.batch * world * args.steps
    value = images / elapsed

    # The headline is BASELINE's metric config, 19 prototypes/class (P = 361). configs[1]/[2]
    # (cityscapes_{no_kld,kld}_imnet.gin) bind 10/class (P = 190): that layer step is reported
    # beside it with its own roofline, and the KLD step runs at P = 190.
    side = None
    if world == 1 and args.side_protos and args.side_protos != args.protos:
        side = LayerStep(args.batch, args.channels, args.fmap, args.fmap, args.side_protos, args.classes, x_dtype,
                         device, SEED + rank, args.precision)
        e_side, k_side, a_side = time_layer(side, args.steps, args.warmup, 1, args.launch == "graph")

    kld = None
    if not args.no_kld and world == 1:
        # configs[2] binds 10 prototypes/class (P = 190); the metric's 19/class beside it. Each
        # against the plain layer step of the same P (ratio_to_plain_step), the dense-g_dist
        # variant as the before/after of the compact gradient.
        kld = {}
        for kstep, e_plain in ((side, e_side if side is not None else None), (step, elapsed)):
            if kstep is None:
                continue
            kstep.setup_kld(SEED + rank)
            line = time_kld_step(kstep, max(5, args.steps // 4), 3)
            dense = time_kld_step(kstep, max(5, args.steps // 4), 3, compact=False)
            line["dense_g_dist_ms_per_step"] = dense["ms_per_step"]
            line["dense_kld_backward_ms"] = dense["kld_backward_ms"]
            line["plain_step_ms"] = round(e_plain / args.steps * 1e3, 4)
            line["ratio_to_plain_step"] = round(line["ms_per_step"] / line["plain_step_ms"], 3)
            kld[f"P{kstep.P}"] = line

    # The same step with exact f32 products (v_mfma_f32_32x32x2_f32, the fma chain of the
    # reference's fp32 conv): what the headline's bf16x3 products trade for their speed.
    exact = None
    if world == 1 and args.precision != "f32" and not args.no_f32_line:
        fstep = LayerStep(args.batch, args.channels, args.fmap, args.fmap, args.protos, args.classes, x_dtype,
                          device, SEED + rank, "f32")
        e_f32, k_f32, a_f32 = time_layer(fstep, max(5, args.steps // 2), 3, 1, args.launch == "graph")
        n_f = max(5, args.steps // 2)
        exact = {"precision": "f32 (exact f32 products, v_mfma_f32_32x32x2_f32)", "prototypes": args.protos,
                 "img_per_s": round(args.batch * n_f / e_f32, 1), "ms_per_step": round(e_f32 / n_f * 1e3, 4),
                 "ratio_to_headline_step": round((e_f32 / n_f) / (elapsed / args.steps), 3),
                 "kernels": {a_f32.get(k, k): {"ms": round(v * 1e3, 4)} for k, v in k_f32.items()}}
        del fstep

    sigmoid = None
    if world == 1 and args.precision == "bf16x3" and args.channels == 64 and not args.no_sigmoid:
        sigmoid = time_sigmoid_step(step, max(5, args.steps // 2), 3)

    push = None
    if not args.no_push:
        push = time_push(args.push_images, args.push_steps, 1, device)
        if world == 1 and args.push_images != 1:  # the 1-image call (push_prototypes(images_per_batch=1))
            one = time_push(1, args.push_steps, 1, device)
            push["images_per_call_1"] = {k: one[k] for k in ("ms_per_img", "argmin_kernel_ms_per_img", "roofline")}

    knn = evaluation = None
    if not args.no_knn and world == 1:
        knn = time_knn(args.push_images, args.push_steps, 1, device)
    if not args.no_eval and world == 1:
        evaluation = time_eval(2, 3, 1, device)
    bboxes = None
    if not args.no_push and world == 1:
        bboxes = time_bound_boxes(3, 1, device)
    small = None
    if not args.no_small_batch and world == 1:
        small = time_small_batches(args, device)
    wide = None
    if not args.no_wide and world == 1:
        # configs[4]: DenseNet-161 add-on depth (BASELINE names a 1024-channel map), 30 prototypes
        # per class x 19 classes, 513x513 crops at output stride 32 -> 16x16 maps, fp16 feature maps
        # (read as fp16 by the GEMM stages, g_x written as fp16); the reference's construct_PPNet default
        # (prototype_shape (2000, 512, 1, 1), 200 classes, 224x224 -> 7x7 maps; model.py:394)
        wide = {"configs4_densenet_c1024_p570": time_wide(device, args.batch, 1024, 16, 16, 570, 19, torch.float16,
                                                          label="configs[4] DenseNet depth, fp16 feature maps"),
                "reference_default_c512_p2000_k200": time_wide(device, args.batch, 512, 7, 7, 2000, 200,
                                                               torch.float32, label="construct_PPNet default")}
    train = None
    if not args.no_train:
        train = time_train_step(args, device, rank, world, args.train_accumulations)

    if rank == 0:
        roof, kernels = layer_report(step, per_kernel, actual, args)
        out = {
            "metric": baseline_metric(),
            "value": round(value, 1),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": f"{args.x_dtype} in; {args.precision} products, f32 accumulate",
            "data": "synthetic (seeded; SURVEY.md §8d shapes), inputs resident in HBM",
            "config": {"workload": f"prototype layer training step: fwd + bwd (+ bucketed RCCL grad all-reduce when N>1) + "
                                   f"Adam update, 513x513 crop -> "
                                   f"{args.fmap}x{args.fmap} map, {args.protos // max(1, args.classes)} prototypes/class "
                                   f"(P={args.protos}, the metric's config), cityscapes_*_imnet.gin otherwise",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "channels": args.channels, "prototypes": args.protos, "classes": args.classes,
                       "parallelism": f"dp{world}", "launch": args.launch},
            "roofline": roof,
            "kernels": kernels,
        }
        if side is not None:
            roof_s, kernels_s = layer_report(side, k_side, a_side, args)
            out[f"protos_{side.P}"] = {
                "prototypes": side.P, "img_per_s": round(args.batch * args.steps / e_side, 1),
                "ms_per_step": round(e_side / args.steps * 1e3, 4),
                "workload": "cityscapes_no_kld_imnet.gin prototype layer training step (10 prototypes/class)",
                "roofline": roof_s, "kernels": kernels_s}
        if sigmoid is not None:
            out["add_on_sigmoid"] = sigmoid
        if exact is not None:
            out["exact_f32"] = exact
        if kld is not None:
            out["kld_step"] = kld
        if push is not None:
            out["push"] = push
        if knn is not None:
            out["knn_search"] = knn
        if evaluation is not None:
            out["eval"] = evaluation
        if bboxes is not None:
            out["push"]["bound_boxes"] = bboxes
        if small is not None:
            out["small_batch"] = small
        if wide is not None:
            out["wide_family"] = wide
        if train is not None:
            out["train_step"] = train
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_layer_baseline(args.batch, args.channels, args.fmap, args.fmap, args.protos,
                                                     args.classes)
            if push is not None:
                out["push"]["cpu_baseline"] = cpu_push_baseline(args.cpu_seconds)
                out["push"]["speedup_vs_cpu"] = round(out["push"]["cpu_baseline"]["ms_per_img"] /
                                                      push["ms_per_img"], 1)
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
