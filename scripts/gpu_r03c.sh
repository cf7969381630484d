set -o pipefail
out=gpurun_out/r03c; mkdir -p $out; export TMPDIR=/tmp
DFQ_CLE_TIMING=1 timeout -k 10 400 python -u scripts/cle_ab.py --reps 5 --configs grouped,grouped_nofence,grouped_nofence_1024,tiles_fin --models mobilenetv2,resnet50 > $out/cle_ab.jsonl 2> $out/cle_ab.err || { echo "cle_ab rc=$?"; tail -30 $out/cle_ab.err; exit 1; }
cat $out/cle_ab.jsonl; grep "group " $out/cle_ab.err | sort | uniq | head -40
