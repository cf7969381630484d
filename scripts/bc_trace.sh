#!/bin/bash
# Kernel trace of the bias-correction chain (run through gpurun from the repo
# root): rocprofv3 --kernel-trace over scripts/bc_host_split.py on one model,
# then the BC kernels' summary and the last replayed chain's dispatches.
set -o pipefail
tag=${1:-bc_trace}
model=${2:-mobilenetv2}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/kt" -o kt -- \
    python3 "$GRAFT_REPO_ROOT/scripts/bc_host_split.py" "$model" > "$GRAFT_REPO_ROOT/$out/bc_split.log" 2>&1 \
    || { echo "bc trace failed rc=$?"; tail -20 "$GRAFT_REPO_ROOT/$out/bc_split.log"; exit 1; }
f=$(find "$GRAFT_REPO_ROOT/$out/kt" -name "*kernel_trace.csv" | head -1)
python3 "$GRAFT_REPO_ROOT/scripts/trace_kernels.py" "$f" --match bc_ --split-us 100 \
    --csv "$GRAFT_REPO_ROOT/$out/bc_chain_$model.csv" > "$GRAFT_REPO_ROOT/$out/summary_$model.txt" 2>&1
cat "$GRAFT_REPO_ROOT/$out/summary_$model.txt"
rm -f "$f"
