#!/bin/bash
# Diagnostics pass (run through gpurun from the repo root): the single-model
# sweep's per-task timeline (variant 13), the specialised vs generic quantize
# loop (variants 6 / 15), the CLE rescale-task timeline
# (DFQ_CLE_TL), the BC stage split, and the per-tensor PMC passes.  Each step has
# its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:-explore}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for m in mobilenetv2 deeplab resnet50; do
  timeout -k 10 120 python -u scripts/timeline.py $m 1 > "$out/timeline_$m.json" 2>&1 \
      || { echo "timeline $m failed"; tail -20 "$out/timeline_$m.json"; exit 1; }
done
timeout -k 10 150 python -u scripts/single_ab.py 6 15 > "$out/single_ab.jsonl" 2>&1 \
    || { echo "single ab failed"; tail -20 "$out/single_ab.jsonl"; exit 1; }
DFQ_LIB=diag DFQ_CLE_TL=1 timeout -k 10 180 python -u scripts/cle_ab.py --configs tiles_fin --models mobilenetv2,resnet50 --reps 1 \
    > "$out/cle_tl.log" 2>&1 || { echo "cle tl failed"; tail -20 "$out/cle_tl.log"; exit 1; }
timeout -k 10 180 python -u scripts/bc_host_split.py > "$out/bc_split.log" 2>&1 || { echo "bc split failed"; tail -20 "$out/bc_split.log"; }
bash scripts/pmc_tensor.sh "$tag/pmc_tensor" > "$out/pmc_tensor.log" 2>&1 || { echo "pmc failed"; tail -20 "$out/pmc_tensor.log"; exit 1; }
echo explore done
