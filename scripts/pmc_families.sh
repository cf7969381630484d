#!/bin/bash
# PMC passes on the sweep kernel for the bench families:
# occupancy / stall / instruction-mix counters per model, one rocprofv3 --pmc
# pass per counter group (never more than 8 SQ / 2 GRBM counters in a pass).
#   bash scripts/pmc_families.sh <tag> [models...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}; shift || true
MODELS=${*:-"resnet50 deeplab mobilenetv2"}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -q -w "$1" $OUT/counters.txt; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
for m in $MODELS; do
  for p in 1 2; do
    eval "want=\$P$p"; use=""
    for c in $want; do if have $c; then use="$use $c"; else echo "skip $c (not listed)"; fi; done
    echo "== $m pass $p:$use"
    timeout -s KILL 120 rocprofv3 --pmc $use --kernel-include-regex sweep_main --output-format csv \
      -d $OUT/${m}_p$p -o pmc -- python3 $R/bench.py --model $m --steps 5 --warmup 1 --cpu-seconds 0 \
      --no-pipeline --no-secondary --no-parity > $OUT/${m}_p$p.log 2>&1
    rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/${m}_p$p.log; exit $rc; fi
  done
done
find $OUT -name "*counter_collection.csv" | head
