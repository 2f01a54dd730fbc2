"""Runs the training backward (protoseg_l2_bwd: g_x, g_P, g_W) a few times at one shape, for
rocprofv3 kernel traces / counter passes. PROTOSEG_BWD (read once by the library) selects the kernel (fused / wave)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import torch  # noqa: E402

from bench import LayerStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--P", type=int, default=361)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fwd", action="store_true", help="also run the forward")
    a = ap.parse_args()
    step = LayerStep(a.B, 64, 65, 65, a.P, 19, torch.float32, "cuda:0", 20220227)
    for _ in range(a.reps):
        if a.fwd:
            step.fwd()
        step.bwd()
    torch.cuda.synchronize()
    print("ok", os.environ.get("PROTOSEG_BWD"), a.P)


if __name__ == "__main__":
    main()
