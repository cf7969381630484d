#!/bin/bash
# One GPU validation pass (run through gpurun from the repo root):
#   1. the GPU test suite      -> gpurun_out/<tag>/pytest_gpu.log
#   2. __graft_entry__.smoke() -> gpurun_out/<tag>/smoke.log
#   3. bench.py (default run)  -> gpurun_out/<tag>/bench.log
#   4. (optional, N2=1) a 2-rank gloo rehearsal of bench.py on the one GPU
# Each step has its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:-validate}
shift || true
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread "$@" \
    > "$out/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$out/pytest_gpu.log"; exit 1; }
tail -3 "$out/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
    || { echo "smoke failed rc=$?"; tail -30 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
timeout -k 10 600 python -u bench.py > "$out/bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -30 "$out/bench.log"; exit 1; }
tail -c 1500 "$out/bench.log"
if [ "${N2:-0}" = "1" ]; then
  DFQ_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 0 \
      --no-pipeline --no-secondary > "$out/bench_n2_gloo.log" 2>&1 || { echo "n2 failed rc=$?"; tail -30 "$out/bench_n2_gloo.log"; exit 1; }
  tail -c 800 "$out/bench_n2_gloo.log"
fi
