#!/bin/bash
export DFQ_LIB=diag   # A/B variants and switches live in libdfq_diag.so
# A/B of persistent-grid sizes (blocks per CU) for sweep variants, one process per setting.
set -u
mkdir -p gpurun_out
for m in ${MODELS:-mobilenetv2 resnet50 deeplab}; do
  for bpc in ${BPCS:-4 5 8 12}; do
    DFQ_SWEEP_BLOCKS_PER_CU=$bpc timeout -k 10 200 python scripts/ab_variants.py --variants ${VARIANTS:-6,9,10} \
      --model $m > gpurun_out/ab_grid_${m}_$bpc.json 2>gpurun_out/ab_grid_${m}_$bpc.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_grid_${m}_$bpc.json'));print('$m bpc=$bpc',{k:(v['algo_GBs'],v['grid']) for k,v in d['variants'].items()})"
  done
done
