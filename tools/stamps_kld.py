"""Per-wave phase timing of kld_partial_kernel from a `make stamps` build, at the bench's KLD shape.

Run on the GPU box: PROTOSEG_HIP_LIB=<csrc>/build_stamps/libprotoseg_hip.so python3 tools/stamps_kld.py [P]
Slots (s_memtime, shader clock, per wave): 0 start, 1 labels + class list + first barrier,
2 class-pixel list built (workgroups with class pixels), 3 first chunk gathered, 4 chunk loop
done, 5 end, 6 end of a workgroup without class pixels; 7 start (s_memrealtime, 100 MHz).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402


def pct(a, qs=(10, 50, 90)):
    return " ".join(f"p{q} {np.percentile(a, q):8.0f}" for q in qs) + f" max {a.max():8.0f}" if len(a) else "none"


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 361
    dev = torch.device("cuda:0")
    B, C, h, w, K = 32, 64, 65, 65, 19
    gen = torch.Generator().manual_seed(0)
    x = torch.sigmoid(2 * torch.randn(B, C, h, w, generator=gen)).to(dev)
    protos = torch.rand(P, C, generator=gen).to(dev)
    wl = (torch.rand(K, P, generator=gen) - 0.5).to(dev)
    blocks = torch.randint(0, K + 1, (B, (h + 7) // 8, (w + 7) // 8), generator=gen)
    tgt = blocks.repeat_interleave(8, 1).repeat_interleave(8, 2)[:, :h, :w].reshape(B, -1).contiguous().to(dev)
    pcls = torch.clamp(torch.arange(P) // (P // K), max=K - 1).to(torch.int32).to(dev)
    mpc = int(torch.bincount(pcls.cpu().long()).max())
    lib = _lib.load()
    lib.protoseg_debug_stamps_kld.restype = ctypes.c_int
    lib.protoseg_debug_stamps_kld.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dist = torch.empty(B, P, h, w, device=dev)
    logits = torch.empty(B, h, w, K, device=dev)
    s = _lib.stream_of(dev)
    P_ = _lib.ptr
    assert lib.protoseg_l2_fwd(P_(x), 0, B, C, h, w, P_(protos), P, P_(wl), K, 1e-4, 0, _lib.PRECISIONS["bf16x3"],
                               P_(dist), None, P_(logits), s) == 0
    kws_b = lib.protoseg_kld_workspace_size(B, P, h * w, K)
    kws = torch.empty(kws_b, device=dev, dtype=torch.uint8)
    kloss = torch.empty((), device=dev)

    def fwd():
        assert lib.protoseg_kld_forward(P_(dist), B, P, h * w, P_(tgt), _lib.I64, P_(pcls), K, mpc, P_(kloss), None,
                                        P_(kws), kws_b, s) == 0

    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    assert lib.protoseg_debug_stamps_kld(None, 0) == 0
    fwd()
    torch.cuda.synchronize()
    buf = np.zeros(1 << 17, dtype=np.uint64)
    assert lib.protoseg_debug_stamps_kld(buf.ctypes.data, buf.nbytes) == 0
    S = (h * w + 1023) // 1024
    n_wg = K * B * S
    st = buf[: n_wg * 4 * 8].reshape(n_wg, 4, 8).astype(np.int64)
    w0 = st[:, 0, :]  # wave 0 of every workgroup
    full = w0[:, 5] > 0
    early = w0[:, 6] > 0
    print(f"P={P} workgroups {n_wg}: with class pixels {full.sum()}, early exit {early.sum()}, "
          f"neither {(~full & ~early).sum()}")
    f = w0[full]
    print("labels+list scan+barrier", pct(f[:, 1] - f[:, 0]))
    print("class-pixel list        ", pct(f[:, 2] - f[:, 1]))
    print("first gather            ", pct(f[:, 3] - f[:, 2]))
    print("chunk loop rest         ", pct(f[:, 4] - f[:, 3]))
    print("reduce + out            ", pct(f[:, 5] - f[:, 4]))
    print("lifetime (pixels)       ", pct(f[:, 5] - f[:, 0]))
    e = w0[early]
    if len(e):
        print("lifetime (early exit)   ", pct(e[:, 6] - e[:, 0]))
    rt = w0[:, 7][w0[:, 7] > 0]
    rt = (rt - rt.min()) * 10  # ns (100 MHz)
    print("start time spread (ns)  ", pct(rt, (10, 25, 50, 75, 90)))


if __name__ == "__main__":
    main()
