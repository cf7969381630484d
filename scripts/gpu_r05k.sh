#!/bin/bash
# Round-5: rotated row-range LDS reads in the sweep -- parity, single-model A/B
# against the previous build, LDS bank-conflict counters on both.
set -o pipefail
tag=${1:-r05k}
out=gpurun_out/$tag
R=$(pwd)
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py tests/test_gpu_bench_workload.py tests/test_gpu_parity_repeat.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -60 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
timeout -k 10 400 python -u scripts/ab_variant_libs.py run 6 norot 6 norot > "$out/single_ab.jsonl" 2>&1 \
    || { echo "ab failed rc=$?"; tail -30 "$out/single_ab.jsonl"; exit 1; }
python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(d['variant'], {r['row']: r.get('graph_us') for r in d.get('baseline_md_rows', [])}, d.get('bench_frac'))
" "$out/single_ab.jsonl"
for lib in - "$R/data_free_quantization_amd/ab/libdfq_vnorot.so"; do
  n=$([ "$lib" = "-" ] && echo rot || echo norot)
  for m in mobilenetv2 resnet50; do
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES \
        --kernel-include-regex sweep_main --output-format csv -d "$R/$out/pmc_${n}_$m" -o pmc \
        -- python3 "$R/scripts/single_pmc.py" "$lib" $m > "$R/$out/pmc_${n}_$m.log" 2>&1) \
        || { echo "pmc $n $m failed rc=$?"; tail -8 "$out/pmc_${n}_$m.log"; exit 1; }
    python - "$out/pmc_${n}_$m" <<'EOF'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(float); n = collections.Counter()
for fn in f:
    for r in csv.DictReader(open(fn)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[1].split("/")[-1], {k: round(v / max(n[k], 1), 1) for k, v in sorted(acc.items())})
EOF
  done
done
