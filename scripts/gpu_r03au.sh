set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03au; mkdir -p $out
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $out/bench.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03au/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print("main", d['value'], d['roofline']['frac'], "parity", d['parity']['mismatches'])
print(json.dumps(d["pipeline_ms"]))
for c in d['secondary_configs']: print(c['config'][:55], c['frac'])
PY
