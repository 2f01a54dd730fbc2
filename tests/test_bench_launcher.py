"""CPU: `bench.py --gpus 2` outside torchrun starts its two ranks itself (torch.distributed.run
as a child process, before any GPU call) and rank 0 prints the one JSON line for the whole job.
--cpu-smoke swaps the GPU step for the gloo gradient exchange, so the launcher runs here."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                          "--cpu-smoke"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    parsed = json.loads(lines[0])
    assert parsed["n_gpus"] == 2
    assert parsed["config"]["parallelism"] == "dp2"
    assert parsed["config"]["backend"] == "gloo"
    assert parsed["config"]["grad_mean_check"] == 1.5  # mean of ranks' 1 and 2: the exchange ran
    assert parsed["steps"] == 3 and parsed["value"] > 0
