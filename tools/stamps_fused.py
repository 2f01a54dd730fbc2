"""Per-wave phase timing of l2_bwd_fused_bf16_kernel from a `make stamps` build.

Run on the GPU box: PROTOSEG_HIP_LIB=<csrc>/build_stamps/libprotoseg_hip.so python3 tools/stamps_fused.py
Slots: 0 start, 1 prologue done, 2 iteration 2 starts (after the barrier); owners: 4 S and g_act
MFMAs done, 5 epilogue + g_s image done, 3 tile done; x waves: 3 tile i+1 converted, 4 tile i+2
loads issued, 5 g_x MFMA loop of tile i-1 done; 6 loop done; 7 start (s_memrealtime).
Cycles are shader clocks (s_memtime).
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
    st = buf.reshape(-1, 8).astype(np.int64)
    wave = np.arange(len(st)) % 8
    live = st[:, 0] != 0
    print(f"waves recorded: {live.sum()}")
    for role, sel in (("owner", live & (wave < 6)), ("x wave", live & (wave >= 6))):
        s = st[sel]
        print(f"-- {role} ({len(s)})")
        print(f"  prologue       {pct(s[:, 1] - s[:, 0])}")
        print(f"  loop total     {pct(s[:, 6] - s[:, 1])}")
        ok = s[:, 2] != 0
        s2 = s[ok]
        if role == "owner":
            print(f"  it2 stage+S+ga {pct(s2[:, 4] - s2[:, 2])}")
            print(f"  it2 epilogue   {pct(s2[:, 5] - s2[:, 4])}")
            print(f"  it2 g_P, g_W   {pct(s2[:, 3] - s2[:, 5])}")
            print(f"  it2 tile       {pct(s2[:, 3] - s2[:, 2])}")
        else:
            print(f"  it2 g_x MFMA   {pct(s2[:, 5] - s2[:, 2])}")
            print(f"  it2 g_x total  {pct(s2[:, 3] - s2[:, 2])}")
    rt = (st[live, 7] - st[live, 7].min()) * 10
    print(f"start (realtime) spread ns: p50 {np.percentile(rt, 50):.0f} max {rt.max():.0f}")


if __name__ == "__main__":
    main()
