export DFQ_LIB=diag   # A/B variants and switches live in libdfq_diag.so
set -u
mkdir -p gpurun_out
for v in 6 1 2 11; do
  DFQ_SWEEP_VARIANT=$v timeout -k 10 120 python scripts/shape_sweep.py "3x3_256x64(row576)" "3x3_256x128(row1152)" "3x3_256x320(row2880)" "3x3_512x512(row4608)" "1x1_256x256" >> gpurun_out/ab3_shape.jsonl 2>gpurun_out/ab3_err_$v.log || exit $?
done
for m in resnet50 deeplab mobilenetv2; do
  timeout -k 10 240 python scripts/ab_variants.py --model $m --variants 6,1,2,11 --rounds 5 > gpurun_out/ab3_$m.json 2>gpurun_out/ab3_err_$m.log || exit $?
done
echo ok
