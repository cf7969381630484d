"""Warm full-DFQ pipeline stage times (ms) on MobileNetV2 and ResNet-50, fastest
of N runs after a warm-up -- the same measurement as bench.py's pipeline_ms."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda:0")
print(json.dumps({m: bench.pipeline_timing(dev, m) for m in sys.argv[1:] or ["mobilenetv2", "resnet50"]}))
