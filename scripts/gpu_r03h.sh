set -o pipefail
export TMPDIR=/tmp
bash scripts/pmc_families.sh r03h_pmc resnet50 deeplab mobilenetv2 > gpurun_out/r03h_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/r03h_pmc.log; exit 1; }
tail -3 gpurun_out/r03h_pmc.log
PROF_TAG=r03h_prof bash scripts/profile.sh > gpurun_out/r03h_prof.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/r03h_prof.log; exit 1; }
tail -3 gpurun_out/r03h_prof.log
