set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03y; mkdir -p $out
DFQ_CLE_TL=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 1 --configs tiles_fin --models resnet50 > $out/cle_tl.log 2>&1 || { echo "tl rc=$?"; tail -30 $out/cle_tl.log; exit 1; }
grep "DFQ_CLE_TL" $out/cle_tl.log | tail -4
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,apply_occ3 > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
grep config $out/cle_ab.jsonl
