set -o pipefail
out=gpurun_out/r03g; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quant.py -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for m in mobilenetv2 resnet50 deeplab; do
  timeout -k 10 300 python -u scripts/ab_variants.py --variants 6,14 --rounds 7 --model $m > $out/ab_$m.json 2>&1 || { echo "ab rc=$?"; tail -20 $out/ab_$m.json; exit 1; }
  tail -3 $out/ab_$m.json
done
timeout -k 10 300 python -u scripts/ab_variants.py --variants 6,14 --rounds 7 --model resnet50 --asym --no-esum > $out/ab_resnet50_asym_noe.json 2>&1 || { echo "ab rc=$?"; exit 1; }
tail -3 $out/ab_resnet50_asym_noe.json
