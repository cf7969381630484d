#!/bin/bash
export DFQ_LIB=diag   # A/B variants and switches live in libdfq_diag.so
# A/B an environment knob on the bench's sweep: ENVS="label:VAR=v,VAR2=w label2:..." BENCH_ARGS="..." REPS=n
# Each configuration runs REPS times, interleaved; one JSON line per run into gpurun_out/ab_env.jsonl.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/ab_env.jsonl; : > $OUT
ARGS="--steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 --no-pipeline --no-secondary ${BENCH_ARGS:-}"
for rep in $(seq ${REPS:-2}); do
  for cfg in $ENVS; do
    label=${cfg%%:*}; envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 120 python bench.py $ARGS > gpurun_out/ab_env_one.log 2>&1 || { echo "fail $label"; tail -5 gpurun_out/ab_env_one.log; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_env_one.log') if l.startswith('{')][-1])
print(json.dumps({'label':'$label','rep':$rep,'algo_GBs':d['roofline']['achieved'],'ms':d['ms_per_step'],'launches':d['roofline']['launches']}))" | tee -a $OUT
  done
done
