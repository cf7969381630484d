#!/bin/bash
export DFQ_LIB=diag   # A/B variants and switches live in libdfq_diag.so
# A/B of the long-row strategies on ResNet-50 and DeepLab (block-row pieces vs reduce launch).
set -u
mkdir -p gpurun_out
for model in resnet50 deeplab; do
  for br in 1 0; do
    DFQ_SWEEP_BLOCKROW=$br timeout -k 10 300 python bench.py --model $model --steps 20 --cpu-seconds 0 \
      --no-pipeline --no-secondary > gpurun_out/ab_${model}_br$br.log 2>&1 || exit $?
    python -c "import json,sys; r=json.loads(open('gpurun_out/ab_${model}_br$br.log').read().strip().splitlines()[-1])['roofline']; print('$model br=$br', r['achieved'], r['launch_ms'], r['launches'], r['grid_blocks'])"
  done
done
