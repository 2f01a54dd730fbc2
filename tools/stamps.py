"""Per-wave phase timing of the bf16 prototype-layer kernels from a `make stamps` build.

Run on the GPU box: PROTOSEG_HIP_LIB=<csrc>/build_stamps/libprotoseg_hip.so python3 tools/stamps.py
Slots (fwd): 0 start, 1 prologue done, 2 tile 1 started (x ready), 3 tile 1 done, 4 full
rounds done, 6 end (remainder tiles done) (s_memtime, shader clock); 7 start (s_memrealtime,
100 MHz, comparable across CUs).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, C, h, w, P, K = int(os.environ.get("B", 32)), 64, 65, 65, int(os.environ.get("P", 190)), 19
    gen = torch.Generator().manual_seed(0)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    wl = (torch.rand(K, P, generator=gen) - 0.5).to(dev)
    dist = torch.empty(B, P, h, w, device=dev)
    logits = torch.empty(B, h, w, K, device=dev)
    lib = _lib.load()
    lib.protoseg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    null = ctypes.c_void_p(None)
    prec = _lib.PRECISIONS[os.environ.get("PREC", "bf16x3")]

    def fwd():
        _lib.call("protoseg_l2_fwd", _lib.ptr(x), 0, B, C, h, w, _lib.ptr(protos), P, _lib.ptr(wl), K, 1e-4, 0, prec,
                  _lib.ptr(dist), null, _lib.ptr(logits), _lib.stream_of(dev))

    for _ in range(3):
        fwd()
    lib.protoseg_debug_stamps(None, 0)
    fwd()
    buf = np.zeros((1 << 17,), dtype=np.uint64)
    assert lib.protoseg_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(-1, 8).astype(np.int64)
    live = st[:, 0] != 0
    st = st[live]
    print(f"waves recorded: {len(st)}")
    rt = (st[:, 7] - st[:, 7].min()) * 10  # ns (100 MHz)
    print(f"start (realtime) spread: p0 {np.percentile(rt, 0):.0f} p50 {np.percentile(rt, 50):.0f} "
          f"p90 {np.percentile(rt, 90):.0f} max {rt.max():.0f} ns")
    names = ["prologue", "x tile 1", "tile 1", "rounds 2+", "-", "remainder"]
    for a in range(6):
        lo, hi = (4, 6) if a == 5 else (a, a + 1)
        d = st[:, hi] - st[:, lo]
        ok = (st[:, hi] != 0) & (st[:, lo] != 0)
        d = d[ok]
        if len(d):
            print(f"{names[a]:14s} cycles: p10 {np.percentile(d, 10):8.0f} p50 {np.percentile(d, 50):8.0f} "
                  f"p90 {np.percentile(d, 90):8.0f} max {d.max():8.0f}")
    tot = st[:, 6] - st[:, 0]
    print(f"{'wave total':14s} cycles: p10 {np.percentile(tot, 10):8.0f} p50 {np.percentile(tot, 50):8.0f} "
          f"p90 {np.percentile(tot, 90):8.0f} max {tot.max():8.0f}")
    # timeline: realtime start vs wave duration (assume ~2.1 GHz shader clock for conversion)
    ends = rt + tot / 2.1
    print(f"approx kernel span {ends.max():.0f} ns; waves starting after 10 us: {(rt > 10000).sum()}")


if __name__ == "__main__":
    main()
