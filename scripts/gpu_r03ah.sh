set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ah; mkdir -p $out
timeout -k 10 300 python -u scripts/pipeline_cprofile.py mobilenetv2 > $out/cprofile.log 2>&1 || { echo "cprofile rc=$?"; tail -20 $out/cprofile.log; exit 1; }
head -4 $out/cprofile.log
