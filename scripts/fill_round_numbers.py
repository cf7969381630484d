"""Fill README.md / DESIGN.md's R05_* placeholders from a bench log (the last
JSON line of `python bench.py`): python scripts/fill_round_numbers.py <bench.log>"""
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
d = [json.loads(ln) for ln in open(sys.argv[1]) if ln.startswith("{")][-1]
sec = {c["config"]: c for c in d["secondary_configs"]}
f = lambda name: "%.3f" % sec[name]["frac"]
rows = {r["row"]: r for r in d["single_model_latency"]["baseline_md_rows"]}
pm = d["pipeline_ms"]["mobilenetv2"]
vals = {
    "R05_HEAD": "%.3f" % d["roofline"]["frac"],
    "R05_R50": f("resnet50 per-ch sym INT8 + clip + BC error sums"),
    "R05_DL": f("deeplab per-ch sym INT8 + clip + BC error sums"),
    "R05_I4": f("resnet50 per-ch asym INT4 + clip"),
    "R05_P4": f("resnet50 per-ch asym INT4 + clip, packed int4 codes"),
    "R05_PT": f("mobilenetv2 per-tensor asym INT8 (quantize_targ_layer) + clip"),
    "R05_PAIR": "%.3f" % [c for c in d["secondary_configs"] if c["config"].startswith("mobilenetv2 bn2 fold")][0]["frac"],
    "R05_SMB": "%.2f" % rows["MobileNetV2 per-channel W8"]["graph_us"],
    "R05_SDL": "%.2f" % rows["DeepLab per-channel W8"]["graph_us"],
    "R05_E2E": "%.2f" % pm["end_to_end"],
    "R05_CLE": "%.2f" % pm["cle"],
    "R05_BC": "%.2f" % pm["bc"],
    "R05_BN1": "%.2f" % pm["bn1"],
}
for name in ("README.md", "DESIGN.md"):
    p = ROOT / name
    s = p.read_text()
    s2 = re.sub(r"R05_[A-Z0-9]+\b", lambda m: vals.get(m.group(0), m.group(0)), s)
    p.write_text(s2)
print(json.dumps(vals))
