#!/bin/bash
# Round-5: observer/forward/BC-edge tests, CLE structure cache, sweep phase
# marks, BN fold split, R50 spread.
set -o pipefail
tag=${1:-r05j}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "tests/test_gpu_pipeline.py::test_compiled_bc_walk_edge_cases" tests/test_gpu_forward.py tests/test_gpu_act_range.py tests/test_gpu_act_fast.py \
    tests/test_gpu_cle_plan.py tests/test_gpu_parity_repeat.py \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
DFQ_CLE_TIMING=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 2 --configs tiles_fin > "$out/plan.log" 2>&1 \
    || { echo "plan print failed rc=$?"; tail -30 "$out/plan.log"; exit 1; }
grep "TIMING create\|python create" "$out/plan.log" | tail -6
timeout -k 10 300 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,no_lag,stop_arrival > "$out/cle_ab.jsonl" 2>&1 \
    || { echo "cle_ab failed rc=$?"; tail -30 "$out/cle_ab.jsonl"; exit 1; }
cat "$out/cle_ab.jsonl"
timeout -k 10 200 python -u scripts/forward_latency.py 32 > "$out/forward.log" 2>&1 \
    || { echo "forward failed rc=$?"; tail -30 "$out/forward.log"; exit 1; }
grep "^{" "$out/forward.log" | head -3
timeout -k 10 120 python -u scripts/timeline.py mobilenetv2 > "$out/timeline_mobilenetv2.json" 2>&1 \
    || { echo "timeline failed rc=$?"; tail -30 "$out/timeline_mobilenetv2.json"; exit 1; }
python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print({k: d[k] for k in ('event_us','span_us','landed_pct','row_params_pct','row_reduce_pct','make_qparams_pct','params_sync_pct','quant_loop_pct','esum_tail_pct','done_pct','whole_row_tasks')})" "$out/timeline_mobilenetv2.json"
timeout -k 10 200 python -u scripts/bn_timing.py > "$out/bn_timing.log" 2>&1 \
    || { echo "bn_timing failed rc=$?"; tail -30 "$out/bn_timing.log"; exit 1; }
grep -v "^DFQ_BN" "$out/bn_timing.log"; grep "^DFQ_BN" "$out/bn_timing.log" | tail -3
timeout -k 10 400 python -u scripts/r50_spread.py 4 > "$out/r50_spread.log" 2>&1 \
    || { echo "r50_spread failed rc=$?"; tail -30 "$out/r50_spread.log"; exit 1; }
tail -1 "$out/r50_spread.log"
