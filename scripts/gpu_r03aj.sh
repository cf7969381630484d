set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03aj; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cle_plan.py -x -v --timeout 120 --timeout-method thread > $out/pytest_cle.log 2>&1 || { echo "pytest cle rc=$?"; tail -40 $out/pytest_cle.log; exit 1; }
tail -1 $out/pytest_cle.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_cli.py tests/test_gpu_parity_repeat.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $out/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03aj/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print(json.dumps(d['pipeline_ms']))
print(json.dumps(d.get('parity')))
PY
