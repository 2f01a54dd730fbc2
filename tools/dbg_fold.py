"""Step-by-step check of the folded layer step (fused Adam + operand prep): eager calls with a
synchronize after each, then graph replays one at a time, printing progress (dbg_fold.py B P
variant)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

B, P, variant = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
os.environ["PROTOSEG_FOLD_PREP"] = "1" if variant == "fold" else "0"
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
s = bench.LayerStep(B, 64, 65, 65, P, 19, torch.float32, dev, bench.SEED)
print(f"B={B} P={P} {variant}: fold={s.fold}", flush=True)
with torch.cuda.stream(stream):
    for i in range(3):
        for name, c in (("fwd", s.fwd), ("bwd", s.bwd), ("opt", s.opt_step)):
            c()
            torch.cuda.synchronize()
            print(f"eager {i} {name} ok (ready={s.ops_ready})", flush=True)
    g = bench.capture(lambda: [s.fwd(), s.bwd(), s.opt_step()], stream)
    print("captured", flush=True)
    for i in range(4):
        g.replay()
        torch.cuda.synchronize()
        print(f"replay {i} ok", flush=True)
print("done", flush=True)
