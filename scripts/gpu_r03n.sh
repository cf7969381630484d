set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03n; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_cle_plan.py tests/test_gpu_pipeline.py tests/test_gpu_parity_repeat.py tests/test_gpu_transforms.py -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,no_self_ranges,no_dw_pairs > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
grep config $out/cle_ab.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$out/trace -o cle -- python /root/repo/scripts/cle_ab.py --reps 2 --configs tiles_fin --models mobilenetv2 > /root/repo/$out/trace.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
