#!/bin/bash
# rocprofv3 passes for the sweep kernel: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (MI355X_MICROARCH.md: they cannot share a pass).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
ARGS="--steps ${STEPS:-20} --warmup 3 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity ${BENCH_ARGS:-}"
run() { local name=$1; shift
  echo "== $name"; timeout -k 10 600 "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "stop"; exit $rc; fi; }
run kt rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py $ARGS
run fetch rocprofv3 --pmc FETCH_SIZE -T --kernel-include-regex sweep_main --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity ${BENCH_ARGS:-}
run write rocprofv3 --pmc WRITE_SIZE -T --kernel-include-regex sweep_main --output-format csv -d $OUT/write -o write -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-pipeline --no-secondary --no-parity ${BENCH_ARGS:-}
find $OUT -name "*.csv" | head -20
