#!/bin/bash
# Same-box A/B of the working tree's product library against the one built from
# the last commit (data_free_quantization_amd/ab/libdfq_vhead.so), after the sweep
# parity tests: single-model rows (graph us) and the bench list's frac.
set -o pipefail
tag=${1:-ab}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py tests/test_gpu_bench_workload.py tests/test_gpu_parity_repeat.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
timeout -k 10 500 python -u scripts/ab_variant_libs.py run 6 head 6 head 6 head > "$out/ab.jsonl" 2>&1 \
    || { echo "ab failed rc=$?"; tail -30 "$out/ab.jsonl"; exit 1; }
python - "$out/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["variant"], {r["row"][:12]: r.get("graph_us") for r in d.get("baseline_md_rows", [])},
              {k: v.get("graph_us") for k, v in d.items() if isinstance(v, dict) and "graph_us" in v},
              d.get("bench_frac"), d.get("error", "")[-300:])
PY
