"""Every CLE diagnostics configuration of tests/test_gpu_parity_repeat.py, one
subprocess each with its own time limit and a progress line per run (diagnostic,
GPU): which configuration, if any, stalls."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {
    "tiles_fin": {}, "tiles_fin_ordered": {"DFQ_CLE_ORDERED": "1"}, "no_dw_pairs": {"DFQ_CLE_NO_DW_PAIRS": "1"},
    "fork": {"DFQ_CLE_FORK": "1"}, "no_self_ranges": {"DFQ_CLE_NO_SELF_RANGES": "1"},
    "apply_occ4": {"DFQ_CLE_APPLY_OCC4": "1"}, "pos_rows16": {"DFQ_CLE_POS_ROWS": "16"},
    "graph": {"DFQ_CLE_GRAPH": "1"}, "batch8": {"DFQ_CLE_BATCH": "8"}, "unfused": {"DFQ_CLE_UNFUSED_FIN": "1"},
    "grouped": {"DFQ_CLE_GROUPS": "1"}, "grouped_40_blocks": {"DFQ_CLE_GROUPS": "1", "DFQ_CLE_GROUP_GRID": "40"},
}
CODE = r"""
import os, sys, time
sys.path.insert(0, os.environ["DFQ_ROOT"])
from tests.parity import pipeline_mismatches
from data_free_quantization_amd import Cross_layer_equal as cle
t = time.time()
r = pipeline_mismatches(sys.argv[1], 8)
print("RUN", sys.argv[1], r["mismatches"], cle.LAST_RUN.get("launched"), round(time.time() - t, 2), flush=True)
"""
for tag, env in CONFIGS.items():
    for name in sys.argv[1:] or ["mobilenetv2"]:
        e = dict(os.environ, DFQ_ROOT=ROOT, DFQ_LIB="diag", DFQ_CLE_STEP_GRID="1000000", DFQ_CLE_MODE="device", **env)
        try:
            r = subprocess.run([sys.executable, "-c", CODE, name], cwd=ROOT, env=e, capture_output=True, text=True,
                               timeout=60)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("RUN")]
            print(tag, name, "rc", r.returncode, line[-1] if line else r.stderr[-500:], flush=True)
            if r.returncode != 0:
                sys.exit(1)
        except subprocess.TimeoutExpired:
            print(tag, name, "TIMEOUT", flush=True)
            sys.exit(2)
