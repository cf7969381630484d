#!/bin/bash
export DFQ_LIB=diag   # A/B variants and switches live in libdfq_diag.so
# Whole-bench A/B (primary + secondary configs + single-model latency) across env
# configurations, interleaved: ENVS="label:VAR=v ..." REPS=n -> gpurun_out/ab_full.jsonl
set -u
mkdir -p gpurun_out
OUT=gpurun_out/ab_full.jsonl; : > $OUT
for rep in $(seq ${REPS:-2}); do
  for cfg in $ENVS; do
    label=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-pipeline > gpurun_out/ab_full_one.log 2>&1 || { echo "fail $label"; tail -5 gpurun_out/ab_full_one.log; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_full_one.log') if l.startswith('{')][-1])
r={'label':'$label','rep':$rep,'primary':d['roofline']['achieved']}
for c in d['secondary_configs']: r[c['config'][:24]]=c['algo_GBs']
for k,v in d['single_model_latency'].items(): r[k+'_us']=v['us']
print(json.dumps(r))" | tee -a $OUT
  done
done
