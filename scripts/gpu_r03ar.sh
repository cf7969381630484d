set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ar; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cle_plan.py tests/test_gpu_pipeline.py tests/test_gpu_parity_repeat.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/cle_async_ab.py product_gate > $out/ab.jsonl 2>&1 || { echo "ab rc=$?"; tail -30 $out/ab.jsonl; exit 1; }
cat $out/ab.jsonl
DFQ_LIB=diag DFQ_CLE_ASYNC_WAIT=value DFQ_AB_MODES=blocking,async timeout -k 10 300 python -u scripts/cle_async_ab.py diag_waitvalue > $out/ab_wv.jsonl 2>&1 || { echo "ab wv rc=$?"; tail -30 $out/ab_wv.jsonl; exit 1; }
cat $out/ab_wv.jsonl
