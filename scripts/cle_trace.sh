#!/bin/bash
# Kernel trace of the CLE device loop (run through gpurun from the repo root):
# rocprofv3 --kernel-trace over scripts/cle_ab.py (product schedule, MobileNetV2
# and ResNet-50, a few warm runs; CONFIG picks a cle_ab configuration), then the
# loop's per-kernel summary.
set -o pipefail
tag=${1:-cle_trace}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
cfg=${CONFIG:-tiles_fin}
for m in ${MODELS:-mobilenetv2 resnet50}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/kt_$m" -o kt -- \
      python3 "$GRAFT_REPO_ROOT/scripts/cle_ab.py" --configs "$cfg" --models "$m" --reps 2 \
      > "$GRAFT_REPO_ROOT/$out/cle_ab_$m.log" 2>&1 || { echo "trace $m failed rc=$?"; tail -20 "$GRAFT_REPO_ROOT/$out/cle_ab_$m.log"; exit 1; }
  f=$(find "$GRAFT_REPO_ROOT/$out/kt_$m" -name "*kernel_trace.csv" | head -1)
  read L N < <(python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(d['launches'], d['iterations'])" "$GRAFT_REPO_ROOT/$out/cle_ab_$m.log")
  python3 "$GRAFT_REPO_ROOT/scripts/cle_trace_summary.py" "$f" --launches "$L" --iterations "$N" \
      --csv "$GRAFT_REPO_ROOT/$out/loop_$m.csv" > "$GRAFT_REPO_ROOT/$out/summary_$m.txt" 2>&1
  cat "$GRAFT_REPO_ROOT/$out/summary_$m.txt"
  rm -f "$f"   # keep the summary and the loop's dispatches, not the multi-MB trace
done
