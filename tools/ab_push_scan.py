"""Interleaved A/B of protoseg_push_update over a SCAN of distinct images (bench.py's push leg:
64 Cityscapes-shaped images in batches, fresh running state per scan), one process: the main
library against every csrc/build_var/*/libprotoseg_hip.so, event-timed per scan; also checks that
every arm leaves the same state.
usage: python tools/ab_push_scan.py [--images 8] [--scan 64] [--protos 190] [--reps 10]"""
import argparse
import ctypes
import glob
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import make_push_inputs  # noqa: E402
from protoseg_amd import _lib  # noqa: E402

CSRC = os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd", "csrc")


def load(path):
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=8)
    ap.add_argument("--scan", type=int, default=64)
    ap.add_argument("--protos", type=int, default=190)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C, H, W, h, w, P, K = 64, 1024, 2048, 129, 257, a.protos, 19
    nb = max(1, a.scan // a.images)
    batches = [make_push_inputs(a.images, C, H, W, h, w, P, K, dev, 20220227 + 1000 * i) for i in range(nb)]
    protos, pc = batches[0][1], batches[0][3]
    arms = {"main": _lib.load()}
    for d in sorted(glob.glob(os.path.join(CSRC, "build_var", "*", "libprotoseg_hip.so"))):
        arms[os.path.basename(os.path.dirname(d))] = load(d)
    s = _lib.stream_of(dev)
    P_ = _lib.ptr

    def fresh():
        return dict(dist=torch.full((P,), math.inf, device=dev), second=torch.full((P,), math.inf, device=dev),
                    img=torch.full((P,), -1, device=dev, dtype=torch.int64),
                    patch=torch.full((P,), -1, device=dev, dtype=torch.int32), fmap=torch.zeros((P, C), device=dev))

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {k: [] for k in arms}
    final = {}
    for rep in range(a.reps + 2):
        for k, lib in arms.items():
            st = fresh()
            torch.cuda.synchronize()
            ev[0].record()
            for i, (x, _, lab, _) in enumerate(batches):
                r = lib.protoseg_push_update(P_(lab), _lib.U8, a.images, H, W, None, 0, 1, P_(x), C, h, w, P_(protos),
                                             P, P_(pc), i * a.images, P_(st["dist"]), P_(st["second"]), P_(st["img"]),
                                             P_(st["patch"]), P_(st["fmap"]), s)
                assert r == 0, lib.protoseg_last_error()
            ev[1].record()
            torch.cuda.synchronize()
            if rep >= 2:
                times[k].append(ev[0].elapsed_time(ev[1]) * 1e3)
            final[k] = st
    n = nb * a.images
    for k, v in times.items():
        med = float(np.median(v))
        print(f"{k:10s} scan of {n} images: median {med:9.1f} us = {med / n:6.2f} us/img  (min {min(v) / n:6.2f})",
              flush=True)
    ref = final["main"]
    for k in arms:
        if k != "main":
            same = all(torch.equal(final[k][f], ref[f]) for f in ref)
            print(f"{k} vs main: state equal {same}")


if __name__ == "__main__":
    main()
