"""Ablation driver for the prototype-layer kernels (run under rocprofv3 --kernel-trace --stats).

Each variant calls the C ABI with some outputs disabled, so per-kernel rocprof times separate
the cost of distance stores, logits, activations and the two backward kernels. Variants are
interleaved in one process (cdna_hip_programming.md §5.4 rule 24). Also prints event timings.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--protos", type=int, default=190)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--precision", default="bf16x3")
    ap.add_argument("--only", default="", help="comma-separated variant names (default: all)")
    ap.add_argument("--fmap", type=int, default=65, help="feature-map side")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B, C, h, w, P, K = args.batch, 64, args.fmap, args.fmap, args.protos, 19
    gen = torch.Generator().manual_seed(0)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    wl = (torch.rand(K, P, generator=gen) - 0.5).to(dev)
    gl = torch.randn(B, h, w, K, generator=gen).to(dev)
    dist = torch.empty(B, P, h, w, device=dev)
    logits = torch.empty(B, h, w, K, device=dev)
    gx = torch.empty_like(x)
    gp = torch.empty(P, C, device=dev)
    gw = torch.empty(K, P, device=dev)
    lib = _lib.load()
    ws_b = lib.protoseg_l2_bwd_workspace_size(B, C, h, w, P, K)
    ws = torch.empty(ws_b, device=dev, dtype=torch.uint8)
    prec = _lib.PRECISIONS[args.precision]
    null = ctypes.c_void_p(None)
    s = lambda: _lib.stream_of(dev)  # noqa: E731
    P_ = _lib.ptr

    variants = {
        "fwd_dist_logits": lambda: _lib.call("protoseg_l2_fwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0,
                                             prec, P_(dist), null, P_(logits), s()),
        "fwd_logits_only": lambda: _lib.call("protoseg_l2_fwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0,
                                             prec, null, null, P_(logits), s()),
        "fwd_dist_only": lambda: _lib.call("protoseg_l2_fwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0,
                                           prec, P_(dist), null, null, s()),
        "fwd_xsig": lambda: _lib.call("protoseg_l2_fwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4,
                                      _lib.X_SIGMOID, prec, P_(dist), null, P_(logits), s()),
        "bwd_full_xsig": lambda: _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4,
                                           _lib.X_SIGMOID, prec, P_(gl), null, P_(gx), P_(gp), P_(gw), P_(ws), ws_b,
                                           s()),
        "fwd_linear": lambda: _lib.call("protoseg_l2_fwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 1,
                                        prec, P_(dist), null, P_(logits), s()),
        "bwd_x_linear": lambda: _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 1,
                                          prec, P_(gl), null, P_(gx), null, null, null, 0, s()),
        "bwd_pw_linear": lambda: _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 1,
                                           prec, P_(gl), null, null, P_(gp), P_(gw), P_(ws), ws_b, s()),
        "bwd_x": lambda: _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, prec,
                                   P_(gl), null, P_(gx), null, null, null, 0, s()),
        "bwd_full": lambda: _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, prec,
                                      P_(gl), null, P_(gx), P_(gp), P_(gw), P_(ws), ws_b, s()),
        "bwd_pw": lambda: _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, prec,
                                    P_(gl), null, null, P_(gp), P_(gw), P_(ws), ws_b, s()),
    }
    if args.only:
        variants = {k: v for k, v in variants.items() if k in args.only.split(",")}
    for fn in variants.values():
        fn()
    torch.cuda.synchronize()
    times = {k: [] for k in variants}
    for _ in range(args.reps):
        for k, fn in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            times[k].append((a, b))
    torch.cuda.synchronize()
    for k, evs in times.items():
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        print(f"{k:18s} median {ms[len(ms) // 2] * 1e3:8.1f} us  min {ms[0] * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
