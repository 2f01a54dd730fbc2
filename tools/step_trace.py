"""One bench step configuration alone, graph-replayed, for a rocprofv3 kernel trace of that
shape: step_trace.py layer|kld [--protos P] [--batch B] [--steps N]. layer: fwd + bwd + Adam
(bench time_layer); kld: fwd + KLD fwd / compact bwd + bwd_kld + Adam (bench time_kld_step)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("what", choices=["layer", "kld"])
ap.add_argument("--protos", type=int, default=361)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--fmap", type=int, default=65)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda:0")
step = bench.LayerStep(args.batch, 64, args.fmap, args.fmap, args.protos, 19, torch.float32, dev, bench.SEED)
calls = [step.fwd, step.bwd, step.opt_step]
if args.what == "kld":
    step.setup_kld(bench.SEED)
    calls = [step.fwd, step.kld_fwd, step.kld_bwd_compact, step.bwd_kld, step.opt_step]
stream = torch.cuda.Stream(dev)
with torch.cuda.stream(stream):
    for _ in range(3):
        for c in calls:
            c()
    torch.cuda.synchronize()
    g = bench.capture(lambda: [c() for c in calls], stream)
    for _ in range(args.steps):
        g.replay()
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.replay()
    torch.cuda.synchronize()
    print(f"{args.what} P={args.protos} B={args.batch}: {(time.perf_counter() - t0) / args.steps * 1e3:.4f} ms/step")
