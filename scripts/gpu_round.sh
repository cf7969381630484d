#!/bin/bash
# One GPU pass for round-4 work (run through gpurun from the repo root):
#   1. bench.py first, on the fresh lease (what the driver measures)
#   2. (optional) a second bench without the time-based pre-warm
#   3. the GPU test suite (or the tests named in $TESTS)
#   4. __graft_entry__.smoke()
# Each step has its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:-round}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 \
      || { echo "bench failed rc=$?"; tail -30 "$out/bench.log"; exit 1; }
  tail -c 600 "$out/bench.log"
fi
if [ "${NOPREWARM:-0}" = "1" ]; then
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --prewarm-ms 0 --no-secondary --no-pipeline \
      --cpu-seconds 0 --no-parity > "$out/bench_noprewarm.log" 2>&1 \
      || { echo "bench (no prewarm) failed rc=$?"; tail -30 "$out/bench_noprewarm.log"; exit 1; }
fi
if [ "${PYTEST:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests -m gpu} -x -v --timeout 280 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$out/pytest_gpu.log"; exit 1; }
  tail -3 "$out/pytest_gpu.log"
fi
if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
      || { echo "smoke failed rc=$?"; tail -30 "$out/smoke.log"; exit 1; }
  tail -2 "$out/smoke.log"
fi
