set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03t; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bc_chain.py -x -q --timeout 120 --timeout-method thread > $out/pytest_bc.log 2>&1 || { echo "pytest bc rc=$?"; tail -60 $out/pytest_bc.log; exit 1; }
tail -1 $out/pytest_bc.log
DFQ_BC_TIMING=1 timeout -k 10 200 python -u scripts/bc_host_split.py > $out/split_coop.log 2>&1 || { echo "split rc=$?"; tail -30 $out/split_coop.log; exit 1; }
DFQ_BC_CHAIN=launches timeout -k 10 200 python -u scripts/bc_host_split.py > $out/split_launches.log 2>&1 || { echo "split rc=$?"; tail -30 $out/split_launches.log; exit 1; }
grep '^{' $out/split_*.log
grep DFQ_BC_TIMING $out/split_coop.log | tail -4
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity > $out/bench_quick.log 2>&1 || { echo "bench rc=$?"; tail -30 $out/bench_quick.log; exit 1; }
tail -c 600 $out/bench_quick.log
