set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03i; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 400 python -u scripts/cle_ab.py --reps 7 --configs tiles_fin,no_dw_pairs,tiles_fin_ordered > $out/cle_ab.jsonl 2>&1 || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.jsonl; exit 1; }
grep config $out/cle_ab.jsonl
bash scripts/pmc_families.sh r03i_pmc resnet50 deeplab mobilenetv2 > $out/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 $out/pmc.log; exit 1; }
PROF_TAG=r03i_prof bash scripts/profile.sh > $out/prof.log 2>&1 || { echo "profile rc=$?"; tail -20 $out/prof.log; exit 1; }
tail -3 $out/prof.log
