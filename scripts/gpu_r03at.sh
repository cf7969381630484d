set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03at; mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --no-parity > $out/bench_nocpu.log 2>&1 || { echo "bench rc=$?"; tail -20 $out/bench_nocpu.log; exit 1; }
grep '^{' $out/bench_nocpu.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('nocpu', json.dumps(d['pipeline_ms']['mobilenetv2']))"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-secondary --no-parity > $out/bench_cpu.log 2>&1 || { echo "bench rc=$?"; tail -20 $out/bench_cpu.log; exit 1; }
grep '^{' $out/bench_cpu.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cpu', json.dumps(d['pipeline_ms']['mobilenetv2']))"
