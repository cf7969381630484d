set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03aq; mkdir -p $out
DFQ_LIB=diag DFQ_CLE_TIMING=1 DFQ_CLE_ASYNC_NOWAIT=1 DFQ_AB_MODES=blocking,async_join_first timeout -k 10 300 python -u scripts/cle_async_ab.py diag_nowait > $out/ab_nowait.log 2>&1 || { echo "ab rc=$?"; tail -30 $out/ab_nowait.log; exit 1; }
grep '^{' $out/ab_nowait.log
grep "loop" $out/ab_nowait.log | head -16
