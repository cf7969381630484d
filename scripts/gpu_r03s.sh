set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03s; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bc_chain.py tests/test_gpu_transforms.py -x -q --timeout 120 --timeout-method thread > $out/pytest_bc.log 2>&1 || { echo "pytest bc rc=$?"; tail -60 $out/pytest_bc.log; exit 1; }
tail -2 $out/pytest_bc.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity_repeat.py tests/test_gpu_cle_plan.py -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 400 python -u scripts/bc_ab.py --reps 7 --configs coop,launches,grid128,grid256 > $out/bc_ab.jsonl 2>&1 || { echo "bc_ab rc=$?"; tail -30 $out/bc_ab.jsonl; exit 1; }
grep config $out/bc_ab.jsonl
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
grep config $out/cle_ab.jsonl
DFQ_BC_TIMELINE=1 timeout -k 10 200 python -u scripts/bc_ab.py --reps 1 --configs coop > $out/bc_timeline.log 2>&1 || { echo "timeline rc=$?"; tail -30 $out/bc_timeline.log; exit 1; }
timeout -k 10 200 python -u scripts/bn_fold_time.py > $out/bn_fold_time.log 2>&1 || { echo "bn rc=$?"; exit 1; }
cat $out/bn_fold_time.log | tail -3
