"""bench.single_model_latency under a kernel trace (run by rocprofv3): the sweep
kernel's own duration per single-model launch vs the per-execute event time."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

dev = torch.device("cuda:0")
print(json.dumps(bench.single_model_latency(dev, torch.cuda.current_stream(dev), reps=50)))
