"""One wide-family layer step configuration from bench.py (for a kernel trace of that shape
alone): wide_run.py c4|ref [steps]. c4: BASELINE configs[4] (DenseNet-161 depth, C = 1024,
P = 570); ref: the reference's construct_PPNet default (C = 512, P = 2000, K = 200)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
prec = sys.argv[3] if len(sys.argv) > 3 else "bf16x3"
dev = torch.device("cuda:0")
if cfg in ("c4", "c4f32"):  # c4: fp16 feature maps as BASELINE states; c4f32: the same in f32
    dt = torch.float16 if cfg == "c4" else torch.float32
    out = bench.time_wide(dev, 32, 1024, 16, 16, 570, 19, dt, steps=steps, label="configs4 " + str(dt), precision=prec)
else:
    out = bench.time_wide(dev, 32, 512, 7, 7, 2000, 200, torch.float32, steps=steps, label="reference default", precision=prec)
print(json.dumps(out))
