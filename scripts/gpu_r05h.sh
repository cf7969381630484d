#!/bin/bash
# Round-5: sweep row-range loads / forward cache / BN fold host split / CLE planner.
set -o pipefail
tag=${1:-r05h}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/single_ab.py 6 15 > "$out/single_ab.jsonl" 2>&1 \
    || { echo "single_ab failed rc=$?"; tail -30 "$out/single_ab.jsonl"; exit 1; }
cat "$out/single_ab.jsonl"
for m in mobilenetv2; do
  timeout -k 10 120 python -u scripts/timeline.py $m > "$out/timeline_$m.json" 2>&1 \
      || { echo "timeline $m failed rc=$?"; tail -30 "$out/timeline_$m.json"; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print({k: d[k] for k in ('model','tasks','event_us','span_us','landed_pct','row_params_pct','quant_loop_pct','esum_tail_pct','done_pct')})" "$out/timeline_$m.json"
done
timeout -k 10 200 python -u scripts/bn_timing.py > "$out/bn_timing.log" 2>&1 \
    || { echo "bn_timing failed rc=$?"; tail -30 "$out/bn_timing.log"; exit 1; }
grep -v "^DFQ_BN" "$out/bn_timing.log"; grep "^DFQ_BN" "$out/bn_timing.log" | tail -4
timeout -k 10 200 python -u scripts/forward_latency.py 32 > "$out/forward.log" 2>&1 \
    || { echo "forward failed rc=$?"; tail -30 "$out/forward.log"; exit 1; }
grep "^{" "$out/forward.log" | head -3
timeout -k 10 900 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_quant.py tests/test_gpu_bench_workload.py \
    tests/test_gpu_pipeline.py -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
DFQ_CLE_TIMING=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 2 --configs tiles_fin > "$out/plan.log" 2>&1 \
    || { echo "plan print failed rc=$?"; tail -30 "$out/plan.log"; exit 1; }
grep "TIMING create" "$out/plan.log" | tail -4
