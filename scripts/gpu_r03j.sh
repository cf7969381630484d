set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03j; mkdir -p $out
DFQ_CLE_TIMING=1 timeout -k 10 300 python -u scripts/cle_ab.py --reps 3 --configs tiles_fin --models mobilenetv2 > $out/cle_timing.jsonl 2> $out/cle_timing.err || { echo "rc=$?"; tail -20 $out/cle_timing.err; exit 1; }
grep -c DFQ_CLE_TIMING $out/cle_timing.err; tail -12 $out/cle_timing.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$out/trace -o cle -- python /root/repo/scripts/cle_ab.py --reps 2 --configs tiles_fin --models mobilenetv2 > /root/repo/$out/trace.log 2>&1 || { echo "rocprof rc=$?"; tail -20 /root/repo/$out/trace.log; exit 1; }
ls /root/repo/$out/trace
