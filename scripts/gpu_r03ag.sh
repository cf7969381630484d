set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ag; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_quant.py tests/test_gpu_bench_workload.py -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/pipeline_cprofile.py mobilenetv2 > $out/cprofile.log 2>&1 || { echo "cprofile rc=$?"; tail -20 $out/cprofile.log; exit 1; }
head -4 $out/cprofile.log
