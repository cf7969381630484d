set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ab; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_cle_plan.py tests/test_gpu_pipeline.py tests/test_gpu_transforms.py tests/test_gpu_parity_repeat.py -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
DFQ_CLE_TL=1 timeout -k 10 200 python -u scripts/cle_ab.py --reps 1 --configs tiles_fin > $out/cle_tl.log 2>&1 || { echo "tl rc=$?"; tail -30 $out/cle_tl.log; exit 1; }
grep "DFQ_CLE_TL step [0-9]:" $out/cle_tl.log | tail -5 | cut -c1-400
timeout -k 10 500 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,apply_occ4,pos_rows16 > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
grep config $out/cle_ab.jsonl
