set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ae; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_transforms.py tests/test_gpu_cle_plan.py tests/test_gpu_bc_chain.py tests/test_gpu_cli.py -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
DFQ_CLE_TIMING=1 timeout -k 10 300 python -u scripts/cle_ab.py --reps 2 --configs tiles_fin --models mobilenetv2 > $out/cle_timing.log 2>&1 || { echo "t rc=$?"; tail -30 $out/cle_timing.log; exit 1; }
grep -v "group" $out/cle_timing.log | grep -E "DFQ_CLE_TIMING|config" | tail -8
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --no-parity > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $out/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03ae/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print(json.dumps(d['pipeline_ms']))
PY
