set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03as; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -30 $out/smoke.log; exit 1; }
tail -3 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $out/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03as/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print("main", d['value'], d['roofline']['frac'], "parity", d['parity']['mismatches'])
print(json.dumps(d['pipeline_ms']['mobilenetv2']), json.dumps(d['pipeline_ms']['resnet50']))
for c in d['secondary_configs']: print(c['config'][:55], c['frac'])
PY
