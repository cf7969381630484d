#!/bin/bash
# Round-5: sweep phase marks, BN fold split, fused observer + forward latency.
set -o pipefail
tag=${1:-r05i}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_act_range.py tests/test_gpu_act_fast.py "tests/test_gpu_pipeline.py::test_compiled_bc_walk_edge_cases" \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
timeout -k 10 200 python -u scripts/forward_latency.py 32 > "$out/forward.log" 2>&1 \
    || { echo "forward failed rc=$?"; tail -30 "$out/forward.log"; exit 1; }
grep "^{" "$out/forward.log" | head -3
for m in mobilenetv2; do
  timeout -k 10 120 python -u scripts/timeline.py $m > "$out/timeline_$m.json" 2>&1 \
      || { echo "timeline $m failed rc=$?"; tail -30 "$out/timeline_$m.json"; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print({k: d[k] for k in ('model','tasks','event_us','span_us','landed_pct','row_params_pct','row_reduce_pct','make_qparams_pct','params_sync_pct','quant_loop_pct','esum_tail_pct','done_pct','whole_row_tasks')})" "$out/timeline_$m.json"
done
timeout -k 10 200 python -u scripts/bn_timing.py > "$out/bn_timing.log" 2>&1 \
    || { echo "bn_timing failed rc=$?"; tail -30 "$out/bn_timing.log"; exit 1; }
grep -v "^DFQ_BN" "$out/bn_timing.log"; grep "^DFQ_BN" "$out/bn_timing.log" | tail -3
