"""bench.fold_quant_pair on its own (main_dfq's bn2 fold + one-pass per-tensor
sweep vs the reduce-pass sweep): one JSON line."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

dev = torch.device("cuda:0")
print(json.dumps(bench.fold_quant_pair(dev, torch.cuda.current_stream(dev))))
