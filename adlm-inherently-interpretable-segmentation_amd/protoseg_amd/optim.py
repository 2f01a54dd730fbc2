"""Adam on the HIP kernel (``protoseg_adam_step``): a drop-in for the reference's optimizer.

Reference: segmentation/module.py:391 builds ``torch.optim.Adam(optimizer_specs)`` (per-group
``lr`` / ``weight_decay``, default betas and eps, amsgrad off). This class takes the same
``params`` / param groups and hyper-parameters and runs each group's update for all its tensors
in one launch (up to 8 tensors per launch). As in torch, every parameter has its own step count
(``state[p]['step']``): it lives on the device ({count, ticket} int32 per parameter) so a HIP
graph holding ``step()`` replays as successive steps, and ``state_dict()`` /
``load_state_dict()`` carry it as torch's float ``step`` scalar, so checkpoints move between this
class and ``torch.optim.Adam`` in both directions. f32 tensors on the GPU only (fails loudly
otherwise).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable

import torch

from . import _lib

_MAX_PER_LAUNCH = 8


class Adam(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._steps: Dict[torch.Tensor, torch.Tensor] = {}
        # parameters layer_step_with_operands already updated for the current iteration: the next
        # step() skips them (and forgets the mark), so step() can follow the fused call for the
        # optimizer's other groups without a second update of the two layer tensors
        self._stepped: Dict[int, torch.Tensor] = {}
        # what the last fused update wrote into which operand block (operands_ready)
        self._operands = None

    def _counter(self, p: torch.Tensor) -> torch.Tensor:
        """Device {step count, ticket} of parameter p, seeded from state[p]['step'] (a loaded
        checkpoint) the first time it is needed."""
        ctr = self._steps.get(p)
        if ctr is None:
            t = self.state[p].get("step", 0)
            t = int(t.item()) if isinstance(t, torch.Tensor) else int(t)
            ctr = torch.tensor([t, 0], dtype=torch.int32, device=p.device)
            self._steps[p] = ctr
        return ctr

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        stepped, self._stepped = self._stepped, {}
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None and stepped.get(id(p)) is not p]
            if not ps:
                continue
            for p in ps:
                _lib.require_device(p, p.grad)
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_contiguous() \
                        or not p.grad.is_contiguous():
                    raise _lib.ProtosegError("protoseg Adam: contiguous float32 parameters and gradients only")
                st = self.state[p]
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                    st.setdefault("step", torch.tensor(0.0))
            b1, b2 = group["betas"]
            for s0 in range(0, len(ps), _MAX_PER_LAUNCH):
                chunk = ps[s0:s0 + _MAX_PER_LAUNCH]
                n = len(chunk)
                keep = [(ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]) for ts in
                        (chunk, [p.grad for p in chunk], [self.state[p]["exp_avg"] for p in chunk],
                         [self.state[p]["exp_avg_sq"] for p in chunk])]
                keep.append((ctypes.c_int64 * n)(*[p.numel() for p in chunk]))
                keep.append((ctypes.c_void_p * n)(*[self._counter(p).data_ptr() for p in chunk]))
                addr = [ctypes.cast(a, ctypes.c_void_p) for a in keep]
                with torch.cuda.device(chunk[0].device):
                    _lib.call("protoseg_adam_step", n, *addr[:5], addr[5], float(group["lr"]), float(b1),
                              float(b2), float(group["eps"]), float(group["weight_decay"]),
                              _lib.stream_of(chunk[0].device))
        return loss

    def _group_of(self, p: torch.Tensor):
        for group in self.param_groups:
            if any(q is p for q in group["params"]):
                return group
        raise _lib.ProtosegError("protoseg Adam: tensor is not one of this optimizer's parameters")

    def _ensure_state(self, p: torch.Tensor):
        st = self.state[p]
        if "exp_avg" not in st:
            st["exp_avg"] = torch.zeros_like(p)
            st["exp_avg_sq"] = torch.zeros_like(p)
            st.setdefault("step", torch.tensor(0.0))
        return st

    @torch.no_grad()
    def layer_step_with_operands(self, protos: torch.Tensor, w_last: torch.Tensor, operands: torch.Tensor,
                                 eps: float, act_kind: int, precision: int) -> bool:
        """step() for the prototype layer's two parameters fused with the next forward's operand
        prep (protoseg_l2_adam_prep): the same updates, plus the images of the updated values in
        ``operands``, so that forward passes ``_lib.OPERANDS_READY`` and launches no prep. Each
        tensor uses its own group's lr / weight_decay (betas and eps must agree). Returns False,
        having run nothing, where the fused entry does not serve the shape or the groups differ in
        betas / eps; the caller then runs a plain forward. Either way the caller runs step() next
        for the rest of the optimizer's parameters (the reference's single joint Adam,
        module.py:391): after a fused update the two layer tensors are marked as stepped for this
        iteration, and that step() skips them."""
        if protos.grad is None or w_last.grad is None:
            return False
        P, C = protos.shape[0], protos[0].numel()
        K = w_last.shape[0]
        gp, gw = self._group_of(protos), self._group_of(w_last)
        if gp["betas"] != gw["betas"] or gp["eps"] != gw["eps"]:
            return False
        lib = _lib.load()
        if not lib.protoseg_l2_adam_prep_supported(C, P, K, precision):
            return False
        for p in (protos, w_last):
            _lib.require_device(p, p.grad)
            if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_contiguous() \
                    or not p.grad.is_contiguous():
                raise _lib.ProtosegError("protoseg Adam: contiguous float32 parameters and gradients only")
        sp, sw = self._ensure_state(protos), self._ensure_state(w_last)
        b1, b2 = gp["betas"]
        with torch.cuda.device(protos.device):
            _lib.call("protoseg_l2_adam_prep", C, P, K, float(eps), int(act_kind), int(precision),
                      _lib.ptr(protos), _lib.ptr(protos.grad), _lib.ptr(sp["exp_avg"]), _lib.ptr(sp["exp_avg_sq"]),
                      _lib.ptr(self._counter(protos)), float(gp["lr"]), float(gp["weight_decay"]),
                      _lib.ptr(w_last), _lib.ptr(w_last.grad), _lib.ptr(sw["exp_avg"]), _lib.ptr(sw["exp_avg_sq"]),
                      _lib.ptr(self._counter(w_last)), float(gw["lr"]), float(gw["weight_decay"]),
                      float(b1), float(b2), float(gp["eps"]), _lib.ptr(operands), operands.numel(),
                      _lib.stream_of(protos.device))
        self._stepped[id(protos)] = protos
        self._stepped[id(w_last)] = w_last
        self._operands = (operands.data_ptr(), operands.numel(), protos, protos._version, protos.data_ptr(), w_last,
                          w_last._version, w_last.data_ptr(), float(eps), int(act_kind), int(precision))
        return True

    def operands_ready(self, protos: torch.Tensor, w_last: torch.Tensor, operands: torch.Tensor, eps: float,
                       act_kind: int, precision: int) -> bool:
        """Whether ``operands`` holds the images of exactly these parameter values for this
        (eps, activation, precision): the last layer_step_with_operands wrote them into this block
        and nothing has changed either tensor since: a tracked in-place write bumps its version
        counter (``push_prototypes``' copy, ``load_state_dict``, another torch optimizer), a new
        ``.data`` tensor moves its address (``prune_prototypes``). Writes through ``.data.copy_``
        are invisible to torch's counter: a caller that writes that way passes ``OPERANDS_READY``
        on its own responsibility. Pass the flag only when this is True."""
        o = self._operands
        return (o is not None and o[0] == operands.data_ptr() and o[1] == operands.numel() and o[2] is protos
                and o[3] == protos._version and o[4] == protos.data_ptr() and o[5] is w_last
                and o[6] == w_last._version and o[7] == w_last.data_ptr()
                and o[8:] == (float(eps), int(act_kind), int(precision)))

    def state_dict(self):
        """torch's layout: state[p] = {'step': float scalar, 'exp_avg', 'exp_avg_sq'} (the step
        copied from the device counter; this synchronises with it)."""
        for p, ctr in self._steps.items():
            self.state[p]["step"] = torch.tensor(float(ctr[0].item()))
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._steps = {}  # re-seeded from the loaded state[p]['step'] at the next step()
