"""Event-timed protoseg_push_argmin alone (8 images 64x129x257, P=190; bench.py's push shape):
median per-launch kernel time over --reps calls. PROTOSEG_HIP_LIB selects a variant build."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from protoseg_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--images", type=int, default=8)
    ap.add_argument("--protos", type=int, default=190)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C, H, W, h, w, K = 64, 1024, 2048, 129, 257, 19
    x, protos, labels, pc = bench.make_push_inputs(a.images, C, H, W, h, w, a.protos, K, dev, bench.SEED)
    from protoseg_amd import push
    mask = push.patch_class_mask(labels, h, w)
    keys = torch.empty((a.images, a.protos), device=dev, dtype=torch.int64)
    second = torch.empty_like(keys)
    st = _lib.stream_of(dev)

    def run():
        _lib.call("protoseg_push_argmin", _lib.ptr(x), a.images, C, h, w, _lib.ptr(protos), a.protos, _lib.ptr(pc),
                  _lib.ptr(mask), _lib.ptr(keys), _lib.ptr(second), st)
    for _ in range(3):
        run()
    t, n = bench.kernel_launch_times("push_argmin", run, a.reps)
    flops = 2.0 * a.images * h * w * a.protos * C
    print(f"{os.environ.get('PROTOSEG_HIP_LIB', 'main')[-60:]:60s} argmin {t * 1e6:8.1f} us/launch x{n} "
          f"{flops / (t * n) / 1e12:6.1f} TF/s ({flops / (t * n) / 1e12 / 157.3:.3f} of f32 MFMA)")


if __name__ == "__main__":
    main()
