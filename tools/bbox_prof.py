"""Times the bound-box kernels at push size: m prototype maps 129x257 -> 1024x2048."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adlm-inherently-interpretable-segmentation_amd"))
import numpy as np
import torch
from protoseg_amd import push

dev = torch.device("cuda:0")
m = int(sys.argv[1]) if len(sys.argv) > 1 else 190
g = torch.Generator(device=dev).manual_seed(0)
d = torch.rand((m, 129, 257), device=dev, generator=g) * 6
y = torch.randint(0, 20, (1, 1024, 2048), device=dev, generator=g).to(torch.uint8)
tc = torch.randint(0, 19, (m,), device=dev, generator=g).to(torch.int32)
r = torch.randint(0, 129, (m,), device=dev, generator=g)
c = torch.randint(0, 257, (m,), device=dev, generator=g)
rf = torch.stack([(r * 1024) // 129, (r * 1024) // 129 + 8, (c * 2048) // 257, (c * 2048) // 257 + 8], 1).to(torch.int32)
for _ in range(2):
    _, up = push.act_upsample(d, 1024, 2048)
    thr, box = push.bound_boxes(up, y, tc, rf)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
reps = 5
e[0].record()
for _ in range(reps):
    _, up = push.act_upsample(d, 1024, 2048)
e[1].record()
for _ in range(reps):
    thr, box = push.bound_boxes(up, y, tc, rf)
e[2].record()
torch.cuda.synchronize()
t_up = e[0].elapsed_time(e[1]) / reps
t_bb = e[1].elapsed_time(e[2]) / reps
gb = m * 1024 * 2048 * 4 / 1e9
print(f"m={m} act_upsample {t_up:.3f} ms ({gb / t_up * 1e3:.0f} GB/s write) bound_boxes {t_bb:.3f} ms "
      f"({t_bb / m * 1e3:.1f} us/prototype); box0 {box[0].tolist()} thr0 {thr[0].item():.5f}")
