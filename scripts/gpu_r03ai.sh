set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ai; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_bc_chain.py tests/test_gpu_cli.py tests/test_gpu_transforms.py -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/pipeline_cprofile.py mobilenetv2 > $out/cprofile.log 2>&1 || { echo "cprofile rc=$?"; tail -20 $out/cprofile.log; exit 1; }
head -4 $out/cprofile.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --no-parity > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $out/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03ai/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print(json.dumps(d['pipeline_ms']))
PY
