"""Times bench.time_bound_boxes alone (P = 190 maps 1024x2048): the push's bound-box post-step."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    print(json.dumps(bench.time_bound_boxes(steps, 2, "cuda")), flush=True)
