"""Interleaved A/B of the layer training step with the operand prep folded into the optimizer
launch (protoseg_l2_adam_prep, 3 launches + reduce) against Adam and the forward's prep as
separate launches (PROTOSEG_FOLD_PREP=0): one HIP graph per variant, replayed alternately on one
box. ab_fold.py [B,P ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

cfgs = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(32, 361), (32, 190), (2, 361), (4, 361)]
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
for B, P in cfgs:
    steps, keep = {}, []  # keep: the graphs point into each LayerStep's buffers
    for name, fold in (("fold", "1"), ("separate", "0")):
        os.environ["PROTOSEG_FOLD_PREP"] = fold
        s = bench.LayerStep(B, 64, 65, 65, P, 19, torch.float32, dev, bench.SEED)
        assert s.fold == (fold == "1"), (name, s.fold)
        keep.append(s)
        with torch.cuda.stream(stream):
            for _ in range(3):
                s.fwd(), s.bwd(), s.opt_step()
            torch.cuda.synchronize()
            steps[name] = bench.capture(lambda s=s: [s.fwd(), s.bwd(), s.opt_step()], stream)
    res = {k: [] for k in steps}
    with torch.cuda.stream(stream):
        for _ in range(7):
            for k, g in steps.items():
                for _ in range(5):
                    g.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(40):
                    g.replay()
                torch.cuda.synchronize()
                res[k].append((time.perf_counter() - t0) / 40 * 1e3)
    print(f"B={B} P={P}: " + ", ".join(f"{k} {np.median(v):.4f} ms (min {min(v):.4f})" for k, v in res.items()),
          flush=True)
