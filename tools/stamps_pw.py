"""Per-wave phase timing of l2_bwd_pw_bf16_kernel from a `make stamps` build (second tile).

Slots: 0 start, 1 prologue issued (image copy + first DMA), 2 tile-1 barrier A passed (raw tile
landed), 3 barrier B passed (split images ready), 5 tile-1 compute done, 6 after the loop; 7 realtime.
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
    gl = torch.randn(B, h, w, K, generator=gen).to(dev)
    gp = torch.empty(P, C, device=dev)
    gw = torch.empty(K, P, device=dev)
    lib = _lib.load()
    lib.protoseg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    ws_b = lib.protoseg_l2_bwd_workspace_size(B, C, h, w, P, K)
    ws = torch.empty(ws_b, device=dev, dtype=torch.uint8)
    null = ctypes.c_void_p(None)

    def pw():
        _lib.call("protoseg_l2_bwd", _lib.ptr(x), 0, B, C, h, w, _lib.ptr(protos), P, _lib.ptr(wl), K, 1e-4, 0, 0,
                  _lib.ptr(gl), null, null, _lib.ptr(gp), _lib.ptr(gw), _lib.ptr(ws), ws_b, _lib.stream_of(dev))

    for _ in range(3):
        pw()
    lib.protoseg_debug_stamps(None, 0)
    pw()
    buf = np.zeros((1 << 17,), dtype=np.uint64)
    assert lib.protoseg_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(-1, 8).astype(np.int64)
    st = st[st[:, 0] != 0]
    print(f"waves recorded: {len(st)}")
    rt = (st[:, 7] - st[:, 7].min()) * 10
    print(f"start spread: p50 {np.percentile(rt, 50):.0f} max {rt.max():.0f} ns")
    phases = [("prologue", 0, 1), ("tile 0 (+wait)", 1, 2), ("convert", 2, 3), ("compute", 3, 5),
              ("remaining tiles", 5, 6)]
    for name, a, b in phases:
        ok = (st[:, b] != 0) & (st[:, a] != 0)
        d = (st[:, b] - st[:, a])[ok]
        if len(d):
            print(f"{name:18s} cycles: p10 {np.percentile(d, 10):8.0f} p50 {np.percentile(d, 50):8.0f} "
                  f"p90 {np.percentile(d, 90):8.0f} max {d.max():8.0f}")
    tot = st[:, 6] - st[:, 0]
    print(f"{'wave total':18s} cycles: p50 {np.percentile(tot, 50):8.0f} max {tot.max():8.0f}")


if __name__ == "__main__":
    main()
