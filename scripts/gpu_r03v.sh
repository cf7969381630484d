set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03v; mkdir -p $out
DFQ_CLE_TL=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 1 --configs tiles_fin > $out/cle_tl.log 2>&1 || { echo "tl rc=$?"; tail -30 $out/cle_tl.log; exit 1; }
grep "DFQ_CLE_TL" $out/cle_tl.log | tail -12
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$out/trace -o cle -- python /root/repo/scripts/cle_ab.py --reps 2 --configs tiles_fin --models mobilenetv2 > /root/repo/$out/trace.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
