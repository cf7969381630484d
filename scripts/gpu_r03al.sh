set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03al; mkdir -p $out
timeout -k 10 900 python -u scripts/cle_diag_configs.py mobilenetv2 || exit $?
