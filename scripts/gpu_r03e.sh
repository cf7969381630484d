set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
bash scripts/pmc_families.sh r03e_pmc resnet50 deeplab mobilenetv2 > gpurun_out/r03e_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/r03e_pmc.log; exit 1; }
tail -5 gpurun_out/r03e_pmc.log
PROF_TAG=r03e_prof bash scripts/profile.sh > gpurun_out/r03e_prof.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/r03e_prof.log; exit 1; }
tail -5 gpurun_out/r03e_prof.log
timeout -k 10 300 python -u scripts/pipeline_cprofile.py mobilenetv2 > gpurun_out/r03e_cprofile.txt 2>&1 || { echo "cprofile rc=$?"; tail -20 gpurun_out/r03e_cprofile.txt; exit 1; }
head -5 gpurun_out/r03e_cprofile.txt
