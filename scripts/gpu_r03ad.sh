set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ad; mkdir -p $out
DFQ_CLE_TIMING=1 timeout -k 10 300 python -u scripts/cle_ab.py --reps 2 --configs tiles_fin > $out/cle_timing.log 2>&1 || { echo "t rc=$?"; tail -30 $out/cle_timing.log; exit 1; }
grep -v "group" $out/cle_timing.log | grep DFQ_CLE_TIMING | tail -12
