set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03v; mkdir -p $out
DFQ_CLE_TL=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 1 --configs tiles_fin > $out/cle_tl.log 2>&1 || { echo "tl rc=$?"; tail -30 $out/cle_tl.log; exit 1; }
grep "DFQ_CLE_TL" $out/cle_tl.log | tail -12
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$out/trace -o cle -- python /root/repo/scripts/cle_ab.py --reps 2 --configs tiles_fin --models mobilenetv2 > /root/repo/$out/trace.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_quant.py tests/test_gpu_pipeline.py tests/test_gpu_bench_workload.py -x -q --timeout 280 --timeout-method thread > $out/pytest_quant.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest_quant.log; exit 1; }
tail -1 $out/pytest_quant.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-pipeline > $out/bench_sec.log 2>&1 || { echo "bench rc=$?"; tail -20 $out/bench_sec.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/r03v/bench_sec.log') if x.startswith('{')][-1]
d=json.loads(l)
print("main", d['roofline']['frac'], "parity", d['parity']['mismatches'] if d.get('parity') else None)
for c in d['secondary_configs']: print(c['config'][:55], c['frac'])
PY
