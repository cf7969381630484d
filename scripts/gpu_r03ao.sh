set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ao; mkdir -p $out
timeout -k 10 300 python -u scripts/cle_async_ab.py product > $out/ab.jsonl 2>&1 || { echo "ab rc=$?"; tail -30 $out/ab.jsonl; exit 1; }
cat $out/ab.jsonl
PROF_TAG=r03ao_prof bash scripts/profile.sh || exit $?
