#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench.  Every GPU step has its
# own time limit; a crash/timeout (anything but pass/fail) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu ${PYTEST_SECS:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --cpu-seconds ${CPU_SECS:-3}
