"""Times protoseg_eval_counts variants at Cityscapes eval size (logits only / + random distances /
+ smooth distances) to split the kernel's time between the argmin loops and the counting."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from protoseg_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
B, H, W, h, w, K, P = 2, 1024, 2048, 129, 257, 19, 190
g = torch.Generator().manual_seed(1)
logits = (torch.randn(B, h, w, K, generator=g) * 3).to(dev)
d_rand = (torch.rand(B, P, h, w, generator=g) * 40).to(dev)
yy, xx = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")
ph = torch.rand(P, 2, generator=g) * 6.28
d_smooth = (20 + 10 * torch.sin(yy[None] / 9 + ph[:, 0, None, None]) * torch.cos(xx[None] / 13 + ph[:, 1, None, None]))
d_smooth = d_smooth[None].repeat(B, 1, 1, 1).contiguous().to(dev)
rng = np.random.default_rng(1)
blocks = rng.integers(0, K + 1, size=(B, H // 16, W // 16)).astype(np.uint8)
anns = torch.from_numpy(np.repeat(np.repeat(blocks, 16, 1), 16, 2)).to(dev)
pc = (torch.arange(P) // 10).to(torch.int32).to(dev)
counts = torch.zeros(2 + 2 * K + P, device=dev, dtype=torch.int64)
null = ctypes.c_void_p(None)
s = _lib.stream_of(dev)


def run(d, n=20):
    def once():
        _lib.call("protoseg_eval_counts", _lib.ptr(logits), _lib.ptr(d), B, h, w, K, P if d is not None else 0,
                  _lib.ptr(anns), _lib.U8, H, W, null, 0, _lib.ptr(pc) if d is not None else null, _lib.ptr(counts), s)
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        once()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n / B * 1e3


print(f"logits only      {run(None):8.1f} us/img")
print(f"+ random dist    {run(d_rand):8.1f} us/img")
print(f"+ smooth dist    {run(d_smooth):8.1f} us/img")
