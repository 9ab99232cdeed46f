"""BASELINE config 3 leg alone (CLUSSL on Foodcom shape), for rocprofv3 kernel traces."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.config3(torch.device("cuda", 0))), flush=True)
