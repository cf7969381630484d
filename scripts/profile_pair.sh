#!/bin/bash
# rocprofv3 passes for main_dfq's bn2 fold + one-pass per-tensor sweep pair
# (scripts/fold_pair.py): kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate PMC passes over the fold and sweep kernels.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-prof_pair}
mkdir -p $OUT
run() { local name=$1; shift
  echo "== $name"; timeout -k 10 300 "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "stop"; exit $rc; fi; }
K='sweep_main|bn_fold_weight'
run kt rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt -- python3 $R/scripts/fold_pair.py
run fetch rocprofv3 --pmc FETCH_SIZE -T --kernel-include-regex $K --output-format csv -d $OUT/fetch -o fetch -- python3 $R/scripts/fold_pair.py
run write rocprofv3 --pmc WRITE_SIZE -T --kernel-include-regex $K --output-format csv -d $OUT/write -o write -- python3 $R/scripts/fold_pair.py
