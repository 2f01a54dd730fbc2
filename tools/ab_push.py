"""Interleaved A/B of the push argmin kernels selected by PROTOSEG_PUSH (wave = the default
wave-streamed kernel, block = the block-staged one) on Cityscapes-shaped maps (bench.py's push
leg: 64 x 129 x 257 f32 maps, 1024 x 2048 u8 labels, P = 190 / 361), kernel-timed with HIP events
around the call (argmin launches + the top-2 fold); also checks that both give the same keys.
usage: python tools/ab_push.py [--images 8] [--protos 190] [--reps 30]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402

CSRC = os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd", "csrc")


def load(path):
    import ctypes
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=8)
    ap.add_argument("--protos", type=int, default=190)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(0)
    n, C, h, w, P, K = a.images, 64, 129, 257, a.protos, 19
    x = torch.sigmoid(2 * torch.randn(n, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    lab = torch.randint(0, K + 1, (n, 1024, 2048), generator=gen, dtype=torch.uint8).to(dev)
    mask = torch.empty((n, h * w), device=dev, dtype=torch.int32)
    pcls = torch.clamp(torch.arange(P) // max(1, P // K), max=K - 1).to(torch.int32).to(dev)
    lib = _lib.load()
    s = _lib.stream_of(dev)
    P_ = _lib.ptr
    assert lib.protoseg_patch_class_mask(P_(lab), _lib.U8, n, 1024, 2048, h, w, None, 0, P_(mask), s) == 0
    import glob
    # arms: the main library's two kernels, plus every build_var/*/libprotoseg_hip.so (wave kernel)
    arms = {"wave": (lib, "wave"), "block": (lib, "block")}
    for d in sorted(glob.glob(os.path.join(CSRC, "build_var", "*", "libprotoseg_hip.so"))):
        arms[os.path.basename(os.path.dirname(d))] = (load(d), "wave")
    keys = {k: torch.empty((n, P), device=dev, dtype=torch.int64) for k in arms}
    second = {k: torch.empty((n, P), device=dev, dtype=torch.int64) for k in arms}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record()
    torch.cuda.synchronize()
    times = {k: [] for k in keys}
    for rep in range(a.reps + 3):
        for k, (lb, mode) in arms.items():
            os.environ["PROTOSEG_PUSH"] = mode
            ev[0].record()
            st = lb.protoseg_push_argmin(P_(x), n, C, h, w, P_(protos), P, P_(pcls), P_(mask), P_(keys[k]),
                                          P_(second[k]), s)
            ev[1].record()
            assert st == 0, lb.protoseg_last_error()
            torch.cuda.synchronize()
            if rep >= 3:
                times[k].append(ev[0].elapsed_time(ev[1]) * 1e3)
    flops = 2.0 * h * w * P * C * n
    for k, v in times.items():
        med = float(np.median(v))
        print(f"{k:6s} median {med:8.1f} us  min {min(v):8.1f} us  {med / n:6.2f} us/img  "
              f"{flops / (med * 1e-6) / 1e12:6.1f} TF/s ({flops / (med * 1e-6) / 157.3e12:.3f} of 157.3)")
    for k in arms:
        if k != "block":
            print(f"{k} vs block: keys equal {bool(torch.equal(keys[k], keys['block']))}, "
                  f"second equal {bool(torch.equal(second[k], second['block']))}")


if __name__ == "__main__":
    main()
