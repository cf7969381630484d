set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03am; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cle_plan.py -x -q --timeout 60 --timeout-method thread > $out/pytest_cle.log 2>&1 || { echo "pytest cle rc=$?"; tail -30 $out/pytest_cle.log; exit 1; }
tail -1 $out/pytest_cle.log
timeout -k 10 300 python -u scripts/cle_async_ab.py product 2>&1 | tee $out/ab.jsonl || exit $?
DFQ_LIB=diag DFQ_CLE_PRIO_NORMAL=1 timeout -k 10 300 python -u scripts/cle_async_ab.py diag_prio_normal 2>&1 | tee -a $out/ab.jsonl || exit $?
