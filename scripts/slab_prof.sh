export DFQ_LIB=diag   # A/B variants and switches live in libdfq_diag.so
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/slab
for mb in ${SLABS:-0 32 64 128}; do
  DFQ_SWEEP_SLAB_MB=$mb timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/slab/s$mb -o s -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-pipeline --no-secondary --granularity tensor --asym --no-esum > gpurun_out/slab/s$mb.log 2>&1 || exit 1
done
find gpurun_out/slab -name "*stats*.csv"
