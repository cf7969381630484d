#!/bin/bash
# Round-5: sweep phase timeline (variant 13 with phase marks) for the single
# models; CLE planner host split; CLE stage A/B.
set -o pipefail
tag=${1:-r05g}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for m in mobilenetv2 deeplab; do
  timeout -k 10 120 python -u scripts/timeline.py $m > "$out/timeline_$m.json" 2>&1 \
      || { echo "timeline $m failed rc=$?"; tail -30 "$out/timeline_$m.json"; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print({k: d[k] for k in ('model','tasks','event_us','span_us','landed_pct','row_params_pct','quant_loop_pct','esum_tail_pct','done_pct')})" "$out/timeline_$m.json"
done
DFQ_CLE_TIMING=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 2 --configs tiles_fin > "$out/plan.log" 2>&1 \
    || { echo "plan print failed rc=$?"; tail -30 "$out/plan.log"; exit 1; }
grep "TIMING create\|python create" "$out/plan.log" | tail -8
timeout -k 10 300 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,no_lag > "$out/cle_ab.jsonl" 2>&1 \
    || { echo "cle_ab failed rc=$?"; tail -30 "$out/cle_ab.jsonl"; exit 1; }
cat "$out/cle_ab.jsonl"
