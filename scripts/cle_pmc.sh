#!/bin/bash
# The CLE loop's HBM traffic (run through gpurun from the repo root): rocprofv3
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (MI355X_MICROARCH.md: they cannot share one), each over scripts/cle_loop_once.py
# (2 blocking runs of the product schedule); then scripts/summarize_cle_pmc.py.
#   bash scripts/cle_pmc.sh <tag> [models...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-cle_pmc}; shift || true
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
run() { local name=$1; shift
  timeout -k 10 120 "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "stop"; exit $rc; fi; }
for m in ${@:-mobilenetv2 resnet50}; do
  run kt_$m rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt_$m -o kt -- python3 $R/scripts/cle_loop_once.py --model $m
  run fetch_$m rocprofv3 --pmc FETCH_SIZE -T --kernel-include-regex cle_loop --output-format csv -d $OUT/fetch_$m -o fetch -- python3 $R/scripts/cle_loop_once.py --model $m
  run write_$m rocprofv3 --pmc WRITE_SIZE -T --kernel-include-regex cle_loop --output-format csv -d $OUT/write_$m -o write -- python3 $R/scripts/cle_loop_once.py --model $m
  find $OUT/kt_$m -name "*kernel_trace.csv" -delete
done
