set -o pipefail
out=gpurun_out/r03d; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cle_plan.py tests/test_gpu_pipeline.py tests/test_gpu_parity_repeat.py tests/test_gpu_cli.py -x -v --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,tiles_fin_ordered,grouped > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
cat $out/cle_ab.jsonl
