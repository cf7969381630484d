set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03u; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 200 python -u scripts/bc_host_split.py > $out/split_launches.log 2>&1 || { echo "split rc=$?"; tail -30 $out/split_launches.log; exit 1; }
grep '^{' $out/split_launches.log
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $out/bench.log; exit 1; }
tail -c 400 $out/bench.log
