set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ap; mkdir -p $out
timeout -k 10 300 python -u scripts/cle_async_ab.py product > $out/ab.jsonl 2>&1 || { echo "ab rc=$?"; tail -30 $out/ab.jsonl; exit 1; }
cat $out/ab.jsonl
DFQ_LIB=diag DFQ_CLE_TIMING=1 timeout -k 10 300 python -u scripts/cle_async_ab.py diag_timing > $out/ab_diag.log 2>&1 || { echo "ab diag rc=$?"; tail -30 $out/ab_diag.log; exit 1; }
grep '^{' $out/ab_diag.log
