"""Per-wave phase timing of l2_bwd_fused_bf16_kernel from a `make stamps` build.

Run on the GPU box: PROTOSEG_HIP_LIB=<csrc>/build_stamps/libprotoseg_hip.so python3 tools/stamps_fused.py
16 slots per wave (FSTAMP in l2_bwd_fused.hip): 0 start, 1 prologue done, 2 iteration 2 starts,
3 iteration 2 work done (before its barrier), 4 after that barrier, 13 loop done, 14 start
(s_memrealtime); owners: 5 convert, 6 stage loads issued, 7 S, 8 g_act, 9 epilogue, 10 split +
g_s image, 11 g_P (+ first g_W); x waves: 6 g_x MFMA loop, 7 stores issued. Shader clocks.
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
    B, C, h, w, P, K = int(os.environ.get("B", 32)), 64, 65, 65, int(os.environ.get("P", 190)), 19
    gen = torch.Generator().manual_seed(0)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    wl = (torch.rand(K, P, generator=gen) - 0.5).to(dev)
    gl = torch.randn(B, h, w, K, generator=gen).to(dev)
    gx = torch.empty_like(x)
    gp = torch.empty(P, C, device=dev)
    gw = torch.empty(K, P, device=dev)
    lib = _lib.load()
    lib.protoseg_debug_stamps_fused.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    ws_b = lib.protoseg_l2_bwd_workspace_size(B, C, h, w, P, K)
    ws = torch.empty(ws_b, device=dev, dtype=torch.uint8)
    null = ctypes.c_void_p(None)
    P_ = _lib.ptr

    def bwd():
        _lib.call("protoseg_l2_bwd", P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, _lib.PRECISIONS["bf16x3"],
                  P_(gl), null, P_(gx), P_(gp), P_(gw), P_(ws), ws_b, _lib.stream_of(dev))

    for _ in range(3):
        bwd()
    lib.protoseg_debug_stamps_fused(None, 0)
    bwd()
    buf = np.zeros((1 << 17,), dtype=np.uint64)
    assert lib.protoseg_debug_stamps_fused(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(-1, 16).astype(np.int64)
    wave = np.arange(len(st)) % 8
    live = st[:, 0] != 0
    print(f"waves recorded: {live.sum()}")

    def seg(s, a, b, name):
        ok = (s[:, a] != 0) & (s[:, b] != 0)
        if ok.any():
            print(f"  {name:16s} {pct(s[ok, b] - s[ok, a])}")

    for role, sel in (("owner", live & (wave < 6)), ("x wave", live & (wave >= 6))):
        s = st[sel]
        print(f"-- {role} ({len(s)})")
        seg(s, 0, 1, "prologue")
        seg(s, 1, 13, "loop total")
        seg(s, 2, 4, "iteration 2")
        seg(s, 3, 4, "it2 barrier wait")
        if role == "owner":
            seg(s, 2, 5, "it2 convert")
            seg(s, 5, 6, "it2 stage issue")
            seg(s, 6, 7, "it2 S")
            seg(s, 7, 8, "it2 g_act")
            seg(s, 8, 9, "it2 epilogue")
            seg(s, 9, 10, "it2 split + g_s")
            seg(s, 10, 11, "it2 g_P+g_W(0)")
            seg(s, 11, 3, "it2 g_W(1) end")
        else:
            seg(s, 2, 6, "it2 g_x MFMA")
            seg(s, 6, 7, "it2 g_x stores")
    rt = (st[live, 14] - st[live, 14].min()) * 10
    print(f"start (realtime) spread ns: p50 {np.percentile(rt, 50):.0f} max {rt.max():.0f}")


if __name__ == "__main__":
    main()
