#!/bin/bash
# Round-5: instruction-fetch counters on the single-model sweep (is the one-task-
# per-wave path waiting on a cold instruction cache?).  One counter block per pass.
set -o pipefail
tag=${1:-r05m}
R=$(pwd)
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
grep -o "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*\|SQ_INSTS_[A-Z_]*" "$out/counters.txt" | sort -u | tr '\n' ' '; echo
have() { grep -q -w "$1" "$out/counters.txt"; }
pass() {   # name counters...
  local name=$1; shift; local use=""
  for c in "$@"; do if have $c; then use="$use $c"; fi; done
  [ -z "$use" ] && { echo "$name: none listed"; return 0; }
  for m in mobilenetv2 resnet50; do
    timeout -s KILL 60 rocprofv3 --pmc $use --kernel-include-regex sweep_main --output-format csv -d "$out/${name}_$m" -o pmc \
      -- python3 "$R/scripts/single_pmc.py" - $m > "$out/${name}_$m.log" 2>&1 || { echo "$name $m rc=$?"; tail -5 "$out/${name}_$m.log"; return 1; }
    python3 - "$out/${name}_$m" <<'EOF'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[1].split("/")[-1], {k: round(v / max(n[k], 1), 1) for k, v in sorted(acc.items())})
EOF
  done
}
pass sq SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_INSTS_SALU && \
pass sqc1 SQC_ICACHE_MISSES SQC_ICACHE_HITS && \
pass sqc2 SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ
