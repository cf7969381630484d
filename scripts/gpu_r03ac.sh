set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ac; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,pos_rows16 > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
grep config $out/cle_ab.jsonl
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $out/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03ac/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print("main", d['value'], d['roofline']['frac'], "parity", d['parity']['mismatches'])
print(json.dumps(d['pipeline_ms']['mobilenetv2']), json.dumps(d['pipeline_ms']['resnet50']))
for c in d['secondary_configs']: print(c['config'][:55], c['frac'])
PY
