"""The bench's push line alone (bench.time_push: push_update over 8 images per call), for a
rocprofv3 kernel trace / counter pass of the push kernels: push_trace.py [n_img] [steps]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
print(json.dumps(bench.time_push(n_img, steps, 3, torch.device("cuda:0"))))
