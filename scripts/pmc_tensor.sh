#!/bin/bash
# PMC passes over the standalone per-tensor sweep (quantize_targ_layer's mode,
# MobileNetV2 x155 per-tensor asym INT8 + clip: a reduce launch, then the
# quantize launch that re-reads every weight) -- kernel trace, FETCH_SIZE,
# WRITE_SIZE, TCC hit / miss, each pass its own run (MI355X_MICROARCH.md).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_tensor}
mkdir -p $OUT
cd /tmp
ARGS="--granularity tensor --asym --no-esum --steps 3 --warmup 1 --prewarm-ms 0 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity"
run() { local name=$1; shift
  timeout -s KILL 120 "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi; }
run kt rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py $ARGS
run fetch rocprofv3 --pmc FETCH_SIZE -T --kernel-include-regex sweep_ --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS
run write rocprofv3 --pmc WRITE_SIZE -T --kernel-include-regex sweep_ --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS
run tcc rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --kernel-include-regex sweep_ --output-format csv -d $OUT/tcc -o tcc -- python3 $R/bench.py $ARGS
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
res = collections.defaultdict(dict)
for name in ("fetch", "write", "tcc"):
    for f in glob.glob(f"{out}/{name}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("dfq::", "")
            acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            res[k][c] = sum(v) / len(v)
for f in glob.glob(f"{out}/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Name"].split("(")[0].replace("dfq::", "")
        if k in res or "sweep" in k:
            res[k]["avg_ns"] = float(r["AverageNs"])
for k, d in res.items():
    if "FETCH_SIZE" in d:
        d["read_bytes_x2"] = d["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in d:
        d["write_bytes"] = d["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in d:
        d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
json.dump(res, open(f"{out}/pmc_tensor.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
