"""CLE step / tile grid caps A/B (diagnostics library, one child process per
setting, interleaved): warm CLE stage ms of the MobileNetV2 pipeline."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
settings = [("2048", "4096"), ("4096", "4096"), ("8192", "4096"), ("16384", "8192"), ("1024", "4096")]
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for sg, tg in settings:
        env = dict(os.environ, DFQ_LIB="diag", DFQ_CLE_STEP_GRID=sg, DFQ_CLE_TILE_GRID=tg)
        r = subprocess.run([sys.executable, str(ROOT / "scripts" / "cold_pipeline.py"), "mobilenetv2", "--preload"],
                           env=env, capture_output=True, text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        d = json.loads(line[-1]) if line else {}
        print(json.dumps({"rep": rep, "step_grid": sg, "tile_grid": tg,
                          "cle_warm_ms": d.get("warm", {}).get("cle"), "cle_cold_ms": d.get("cold", {}).get("cle")}),
              flush=True)
