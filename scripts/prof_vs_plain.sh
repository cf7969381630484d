#!/bin/bash
set -o pipefail
# Same box, same command: the headline bench plain, under rocprofv3 --kernel-trace
# --stats, and plain again (is a profiled launch slower than an unprofiled one?).
mkdir -p gpurun_out/r05ak
export TMPDIR=/tmp
A="--steps 20 --warmup 3 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity"
timeout -k 10 200 python3 bench.py $A > gpurun_out/r05ak/plain1.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05ak/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/gpurun_out/r05ak/prof.log 2>&1) || exit 1
timeout -k 10 200 python3 bench.py $A > gpurun_out/r05ak/plain2.log 2>&1 || exit 1
for f in plain1 prof plain2; do python3 -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print(sys.argv[2], d['roofline']['launch_ms'], d['roofline']['frac'])" gpurun_out/r05ak/$f.log $f; done
