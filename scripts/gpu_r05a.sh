#!/bin/bash
# Round-5 GPU pass: the CLE pacing loop without per-iteration hipStreamQuery
# (kernel trace + stage timing), then the CLE plan tests and the N=2 bench test.
set -o pipefail
tag=${1:-r05a}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
MODELS=mobilenetv2 CONFIG=tiles_fin timeout -k 10 300 bash scripts/cle_trace.sh "$tag/trace" \
    > "$out/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -30 "$out/trace.log"; exit 1; }
cat "$out/trace.log"
timeout -k 10 300 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,blocking > "$out/cle_ab.jsonl" 2>&1 \
    || { echo "cle_ab failed rc=$?"; tail -30 "$out/cle_ab.jsonl"; exit 1; }
cat "$out/cle_ab.jsonl"
timeout -k 10 600 python -u -m pytest tests/test_gpu_cle_plan.py tests/test_bench_launcher.py -m gpu -x -v \
    --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -5 "$out/pytest.log"
