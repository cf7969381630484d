#!/bin/bash
# Round-5: packed-math quantize loop -- parity on the sweep / pipeline tests, the
# single-model rows, the ablation table and a short bench.
set -o pipefail
tag=${1:-r05u}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py tests/test_gpu_bench_workload.py tests/test_gpu_parity_repeat.py \
    tests/test_gpu_pipeline.py tests/test_gpu_transforms.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
timeout -k 10 200 python -u scripts/single_ablate.py mobilenetv2 deeplab > "$out/ablate.jsonl" 2>&1 \
    || { echo "ablate failed rc=$?"; tail -30 "$out/ablate.jsonl"; exit 1; }
grep "^{" "$out/ablate.jsonl"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 \
    || { echo "bench failed rc=$?"; tail -30 "$out/bench.log"; exit 1; }
python - "$out/bench.log" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["frac"], d.get("parity"))
print(d["single_model_latency"]["baseline_md_rows"])
print({k: v.get("graph_us") for k, v in d["single_model_latency"].items() if isinstance(v, dict)})
PY
