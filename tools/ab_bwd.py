"""Interleaved A/B of the training-backward kernels selected by protoseg_set_backward_kernel
(wave / fused) at one shape, in one process: per rep, each kernel's forward + backward call on its own
LayerStep (same seed, same inputs), the backward call timed with HIP events and the backward
kernel alone with the library's per-launch event hook. Also checks that the gradients agree.
usage: python tools/ab_bwd.py --protos 190 --batch 32 --kernels fused,wave [--reps 30]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import LayerStep  # noqa: E402
from protoseg_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--protos", type=int, default=361)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--fmap", type=int, default=65)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--kernels", default="fused,wave")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    kernels = a.kernels.split(",")
    steps = {}
    for k in kernels:
        _lib.call("protoseg_set_backward_kernel", k.encode())
        steps[k] = LayerStep(a.batch, 64, a.fmap, a.fmap, a.protos, 19, torch.float32, dev, 20220227)
    lib = _lib.load()
    s = torch.cuda.Stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(s):
        for e in ev + kev:
            e.record(s)
        torch.cuda.synchronize()
        starts = (ctypes.c_void_p * 1)(kev[0].cuda_event)
        stops = (ctypes.c_void_p * 1)(kev[1].cuda_event)
        call, kern = {k: [] for k in kernels}, {k: [] for k in kernels}
        for rep in range(a.reps + 3):
            for k in kernels:
                _lib.call("protoseg_set_backward_kernel", k.encode())
                st = steps[k]
                st.fwd()
                ev[0].record(s)
                st.bwd()
                ev[1].record(s)
                torch.cuda.synchronize()
                if rep >= 3:
                    call[k].append(ev[0].elapsed_time(ev[1]) * 1e3)
                lib.protoseg_timing_events_n(b"l2_bwd", starts, stops, 1)
                try:
                    lib.protoseg_timing_launches()
                    st.bwd()
                    torch.cuda.synchronize()
                    if rep >= 3:
                        kern[k].append(kev[0].elapsed_time(kev[1]) * 1e3)
                    name = lib.protoseg_timing_kernel().decode()
                finally:
                    lib.protoseg_timing_events_n(None, None, None, 0)
                if rep == 3:
                    print(f"{k}: kernel {name}", flush=True)
    for k in kernels:
        print(f"{k:8s} call median {np.median(call[k]):8.2f} us  kernel median {np.median(kern[k]):8.2f} us "
              f"(min {np.min(kern[k]):.2f})", flush=True)
    ref = steps[kernels[0]]
    for k in kernels[1:]:
        o = steps[k]
        for name, u, v in (("g_x", ref.g_x, o.g_x), ("g_p", ref.g_p, o.g_p), ("g_w", ref.g_w, o.g_w)):
            scale = u.abs().max().item() + 1e-30
            err = (u - v).abs().max().item()
            print(f"{k} vs {kernels[0]} {name}: max err {err:.3e} / scale {scale:.3e} = {err / scale:.2e}")


if __name__ == "__main__":
    main()
