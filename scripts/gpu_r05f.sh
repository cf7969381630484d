#!/bin/bash
# Round-5: sweep quantize loop with batched LDS loads + DPP row reductions:
# single-model A/B (v6 vs the generic loop v15), sweep parity tests, the bench,
# and the CLE planner's host split.
set -o pipefail
tag=${1:-r05f}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/single_ab.py 6 15 > "$out/single_ab.jsonl" 2>&1 \
    || { echo "single_ab failed rc=$?"; tail -30 "$out/single_ab.jsonl"; exit 1; }
cat "$out/single_ab.jsonl"
timeout -k 10 900 python -u -m pytest tests/test_gpu_quant.py tests/test_gpu_bench_workload.py tests/test_gpu_pipeline.py \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
DFQ_CLE_TIMING=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 2 --configs tiles_fin > "$out/plan.log" 2>&1 \
    || { echo "plan print failed rc=$?"; tail -30 "$out/plan.log"; exit 1; }
grep "TIMING create" "$out/plan.log" | tail -4
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/bench.log" 2>&1 \
    || { echo "bench failed rc=$?"; tail -30 "$out/bench.log"; exit 1; }
python - "$out/bench.log" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print("value", d["value"], "frac", d["roofline"]["frac"], "parity", d["parity"]["mismatches"])
print(d["single_model_latency"]["baseline_md_rows"])
print({k: d["pipeline_ms"]["mobilenetv2"][k] for k in ("bn1", "cle", "bc", "total", "end_to_end")})
for s in d["secondary_configs"]: print(s["config"][:40], s["frac"])
PY
