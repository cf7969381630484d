#!/bin/bash
# Why boxes differ (diagnostic, GPU): the headline launch time on this box, then
# address-translation and memory-queue counters of the same command, one
# rocprofv3 --pmc pass per counter group (<= 4 TCP / 4 TCC counters a pass).
#   bash scripts/box_probe.sh <tag>
set -o pipefail
tag=${1:-box}
R=$(pwd)
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
A="--steps 10 --warmup 3 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity"
timeout -k 10 200 python3 bench.py $A > "$out/plain.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$out/plain.log"; exit 1; }
python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
t=[s for s in d['timing']['telemetry'] if s['tag']=='after_timed'][0]
print('launch_ms', d['roofline']['launch_ms'], 'frac', d['roofline']['frac'], 'umc', t.get('average_umc_activity'), 'mem_C', t.get('temperature_mem'))" "$out/plain.log"
pass() {
  local name=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex sweep_main --output-format csv \
      -d "$out/$name" -o pmc -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-pipeline \
      --no-secondary --no-parity > "$out/$name.log" 2>&1) || { echo "$name rc=$?"; tail -5 "$out/$name.log"; return 1; }
  python3 - "$out/$name" <<'EOF'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[1].split("/")[-1], {k: round(v / max(n[k], 1)) for k, v in sorted(acc.items())})
EOF
}
pass utcl TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_PENDING_STALL_CYCLES && \
pass ea TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ TCC_EA0_WRREQ_LEVEL && \
pass stall TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL TCC_TAG_STALL
