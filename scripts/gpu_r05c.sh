#!/bin/bash
# Round-5: the lagged CLE schedule -- placement print, stage timing A/B,
# CLE / pipeline parity tests, kernel trace.
set -o pipefail
tag=${1:-r05c}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
DFQ_CLE_TIMING=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 1 --configs tiles_fin > "$out/plan.log" 2>&1 \
    || { echo "plan print failed rc=$?"; tail -30 "$out/plan.log"; exit 1; }
grep "plan:" "$out/plan.log" | sort | uniq -c
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs ${CONFIGS:-tiles_fin,no_lag,band1,band2,blocking} > "$out/cle_ab.jsonl" 2>&1 \
    || { echo "cle_ab failed rc=$?"; tail -30 "$out/cle_ab.jsonl"; exit 1; }
cat "$out/cle_ab.jsonl"
timeout -k 10 900 python -u -m pytest tests/test_gpu_cle_plan.py tests/test_gpu_parity_repeat.py tests/test_gpu_pipeline.py \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
MODELS=${TRACE_MODELS:-mobilenetv2} CONFIG=tiles_fin timeout -k 10 300 bash scripts/cle_trace.sh "$tag/trace" \
    > "$out/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -30 "$out/trace.log"; exit 1; }
cat "$out/trace.log"
