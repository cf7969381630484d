#!/bin/bash
# Task-size A/B of the sweep (diagnostics variants 6 = 2048, 10 = 1536, 12 = 1792
# elements per wave task) on the three bench families and the single-model rows,
# with this box's headline frac for context.
set -o pipefail
tag=${1:-chunk}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 100 python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity > "$out/plain.log" 2>&1 || exit 1
python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print('box frac', d['roofline']['frac'])" "$out/plain.log"
for m in mobilenetv2 resnet50 deeplab; do
  timeout -k 10 300 python3 scripts/ab_variants.py --model $m --variants 6,10,12 --rounds 5 > "$out/ab_$m.log" 2>&1 || { tail -5 "$out/ab_$m.log"; exit 1; }
  python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print(sys.argv[2], {v: r['frac'] for v, r in d['variants'].items()})" "$out/ab_$m.log" $m
done
DFQ_SINGLE_ESUM=0 timeout -k 10 200 python3 scripts/single_ab.py 6 10 12 6 10 12 > "$out/single.log" 2>&1 || { tail -5 "$out/single.log"; exit 1; }
grep "^{" "$out/single.log"
