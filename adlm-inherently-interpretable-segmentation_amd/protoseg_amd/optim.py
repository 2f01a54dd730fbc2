"""Adam on the HIP kernel (``protoseg_adam_step``): a drop-in for the reference's optimizer.

Reference: segmentation/module.py:391 builds ``torch.optim.Adam(optimizer_specs)`` (per-group
``lr`` / ``weight_decay``, default betas and eps, amsgrad off). This class takes the same
``params`` / param groups and hyper-parameters and runs each group's update for all its tensors
in one launch (up to 8 tensors per launch), with the step count on the device so a HIP graph
holding ``step()`` replays as successive steps. f32 tensors on the GPU only (fails loudly
otherwise).
"""
from __future__ import annotations

import ctypes
from typing import Iterable

import torch

from . import _lib

_MAX_PER_LAUNCH = 8


class Adam(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._state_dev = {}

    def _group_state(self, gi: int, device) -> torch.Tensor:
        st = self._state_dev.get(gi)
        if st is None:
            st = torch.zeros(2, dtype=torch.int32, device=device)  # {step count, ticket}
            self._state_dev[gi] = st
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                _lib.require_device(p, p.grad)
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_contiguous() \
                        or not p.grad.is_contiguous():
                    raise _lib.ProtosegError("protoseg Adam: contiguous float32 parameters and gradients only")
                st = self.state[p]
                if not st:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
            dev_state = self._group_state(gi, ps[0].device)
            b1, b2 = group["betas"]
            # Tensors of one group share the step count: one launch per <= 8 tensors, the step
            # count advanced by the first launch only (later launches of the group read it back).
            for s0 in range(0, len(ps), _MAX_PER_LAUNCH):
                chunk = ps[s0:s0 + _MAX_PER_LAUNCH]
                n = len(chunk)
                keep = [(ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]) for ts in
                        (chunk, [p.grad for p in chunk], [self.state[p]["exp_avg"] for p in chunk],
                         [self.state[p]["exp_avg_sq"] for p in chunk])]
                keep.append((ctypes.c_int64 * n)(*[p.numel() for p in chunk]))
                addr = [ctypes.cast(a, ctypes.c_void_p) for a in keep]
                st_t = dev_state if s0 == 0 else self._replay_state(gi, dev_state)
                with torch.cuda.device(chunk[0].device):
                    _lib.call("protoseg_adam_step", n, *addr, _lib.ptr(st_t), float(group["lr"]), float(b1),
                              float(b2), float(group["eps"]), float(group["weight_decay"]),
                              _lib.stream_of(chunk[0].device))
        return loss

    def _replay_state(self, gi: int, advanced: torch.Tensor) -> torch.Tensor:
        """For a group's 2nd+ launch: {t - 1, 0}, so it uses the same step t as the first."""
        key = ("r", gi)
        st = self._state_dev.get(key)
        if st is None:
            st = torch.zeros(2, dtype=torch.int32, device=advanced.device)
            self._state_dev[key] = st
        st[0].copy_(advanced[0] - 1)
        st[1].zero_()
        return st
