#!/bin/bash
# Single-model sweep kernel durations as rocprofv3 sees them (diagnostic, GPU):
# BASELINE.md's W8 rows (one weight set, per-channel W8 + codes, no E), 20
# executes each, kernel trace + stats.  The bench's single_model_latency reports
# kernel-to-kernel time from HIP-graph replays, which includes the ~1.7 us
# dispatch boundary; this is the kernel's own duration.
set -o pipefail
R=$(pwd)
out=$R/gpurun_out/${1:-single_prof}
mkdir -p "$out"
export TMPDIR=/tmp
for m in mobilenetv2 deeplab resnet50; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$m" -o kt \
      -- python3 "$R/scripts/single_pmc.py" - $m w8 > "$out/$m.log" 2>&1) || { echo "$m rc=$?"; tail -5 "$out/$m.log"; exit 1; }
  python3 - "$out/$m" $m <<'PY'
import csv, glob, sys, statistics
f = glob.glob(sys.argv[1] + "/**/kt_kernel_trace.csv", recursive=True)[0]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f)) if "sweep_main" in r["Kernel_Name"]]
d = d[5:]
print(sys.argv[2], "launches", len(d), "median_us", round(statistics.median(d) / 1e3, 2), "min_us", round(min(d) / 1e3, 2))
PY
done
