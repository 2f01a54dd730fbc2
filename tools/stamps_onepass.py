"""Per-wave phase timing of l2_bwd_onepass_bf16_kernel from a `make stamps` build.

Run on the GPU box: PROTOSEG_HIP_LIB=<csrc>/build_stamps/libprotoseg_hip.so PROTOSEG_BWD=onepass
python3 tools/stamps_onepass.py. Slots (OSTAMP in l2_bwd_onepass.hip, iteration 2): 0 start,
1 prologue done, 2 iteration starts, 3/4/5 owner tiles 0/1/2 done, 6 after barrier 1, 7 phase B
MFMAs issued (loads of the next tile issued before), 8 staging done, 9 after barrier 2,
10 epilogue done, 13 loop done. Shader clocks.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402


def pct(d):
    return f"p10 {np.percentile(d, 10):8.0f} p50 {np.percentile(d, 50):8.0f} p90 {np.percentile(d, 90):8.0f} max {d.max():8.0f}"


def main():
    dev = torch.device("cuda:0")
    B, C, h, w, P, K = int(os.environ.get("B", 32)), 64, 65, 65, int(os.environ.get("P", 361)), 19
    gen = torch.Generator().manual_seed(0)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    wl = (torch.rand(K, P, generator=gen) - 0.5).to(dev)
    gl = torch.randn(B, h, w, K, generator=gen).to(dev)
    gx = torch.empty_like(x)
    gp = torch.empty(P, C, device=dev)
    gw = torch.empty(K, P, device=dev)
    lib = _lib.load()
    lib.protoseg_debug_stamps_onepass.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    ws_b = lib.protoseg_l2_bwd_workspace_size(B, C, h, w, P, K)
    ws = torch.empty(ws_b, device=dev, dtype=torch.uint8)
    null = ctypes.c_void_p(None)
    P_ = _lib.ptr

    def bwd():
        _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, _lib.PRECISIONS["bf16x3"],
                  P_(gl), null, P_(gx), P_(gp), P_(gw), P_(ws), ws_b, _lib.stream_of(dev))

    for _ in range(3):
        bwd()
    lib.protoseg_debug_stamps_onepass(None, 0)
    bwd()
    buf = np.zeros((1 << 17,), dtype=np.uint64)
    assert lib.protoseg_debug_stamps_onepass(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(-1, 16).astype(np.int64)
    live = st[:, 0] != 0
    s = st[live]
    print(f"waves recorded: {len(s)} (P={P})")

    def seg(a, b, name):
        ok = (s[:, a] != 0) & (s[:, b] != 0)
        if ok.any():
            print(f"  {name:18s} {pct(s[ok, b] - s[ok, a])}")

    seg(0, 1, "prologue")
    seg(1, 13, "loop total")
    seg(2, 10, "iteration 2")
    seg(2, 3, "owner tile 0")
    seg(3, 4, "owner tile 1")
    seg(4, 5, "owner tile 2")
    seg(5, 6, "barrier 1 wait")
    seg(6, 7, "phase B")
    seg(7, 8, "staging")
    seg(8, 9, "barrier 2 wait")
    seg(9, 10, "g_x epilogue")
    # by wave index in the workgroup (waves w and w + 4 share a SIMD): p50 cycles
    widx = np.nonzero(live)[0] % 8
    print("  wave  owner A  barrier1  phase B  staging  barrier2")
    for wv in range(8):
        r = s[widx == wv]
        ok = (r[:, 2] != 0) & (r[:, 10] != 0)
        r = r[ok]
        if len(r):
            p50 = lambda a, b: np.percentile(r[:, b] - r[:, a], 50)
            print(f"  {wv:4d} {p50(2, 5):8.0f} {p50(5, 6):9.0f} {p50(6, 7):8.0f} {p50(7, 8):8.0f} {p50(8, 9):9.0f}")


if __name__ == "__main__":
    main()
